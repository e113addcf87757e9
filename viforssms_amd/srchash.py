"""Source hash of libvissm.so: sha256 over the library's sources (csrc/*.hip, csrc/*.hpp, csrc/Makefile,
include/vissm.h), each as its path relative to the repo root, a NUL, its bytes and a NUL, in sorted path order.

The Makefile compiles this hash into the library (vissm_source_hash); `_lib.load()` recomputes it from the tree
it runs in and refuses a library built from other sources -- a stale `.so` pushed to a GPU box cannot become the
tested binary.  No torch import: the Makefile runs this file as a script."""
import glob
import hashlib
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_PKG)


def source_files(root: str = _ROOT) -> list:
    csrc = os.path.join(root, "viforssms_amd", "csrc")
    files = glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp"))
    files += [os.path.join(csrc, "Makefile"), os.path.join(root, "include", "vissm.h")]
    return sorted(os.path.relpath(f, root) for f in files)


def source_hash(root: str = _ROOT) -> str:
    h = hashlib.sha256()
    for rel in source_files(root):
        h.update(rel.encode() + b"\0")
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()


if __name__ == "__main__":
    print(source_hash())
