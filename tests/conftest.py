import faulthandler
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

_T0 = time.time()
_FH_FILE = None


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the libvissm HIP kernels)")


def pytest_sessionstart(session):
    """A fatal signal (SIGABRT from the HIP runtime, SIGSEGV) dumps the CURRENT thread's Python stack into
    gpurun_out/faulthandler.log instead of the all-threads dump + extension-module list pytest writes to stderr,
    which is longer than the tail a driver keeps: the last `[vissm-test]` line on stderr names the test."""
    global _FH_FILE
    try:
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        _FH_FILE = open(os.path.join(ROOT, "gpurun_out", "faulthandler.log"), "w")
        faulthandler.enable(file=_FH_FILE, all_threads=False)
    except OSError:
        faulthandler.enable(all_threads=False)


def pytest_runtest_logstart(nodeid, location):
    if os.environ.get("VISSM_TEST_TRACE", "1") != "0":
        sys.__stderr__.write(f"[vissm-test {time.time() - _T0:7.1f}s] {nodeid}\n")
        sys.__stderr__.flush()
