"""Drop-in for the reference's optimisers/adamax.py (implementation: viforssms_amd/optim.py)."""
from viforssms_amd.optim import AdamaxOptimizer  # noqa: F401
