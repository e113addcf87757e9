"""viforssms_amd: MI355X-native neural-moving-average variational inference for SDEs.

The per-transition hot path (IAF flows, ELBO log-densities, clip + Adamax) runs in
hand-written gfx950 HIP kernels (libvissm.so, C ABI in include/vissm.h); this
package is the Python host that mirrors the reference's API (VI_SSM, AR.main,
data_gen, AdamaxOptimizer).
"""
from ._lib import load as load_library, VissmError  # noqa: F401

__version__ = "0.1.0"
