"""Drop-in for the reference's SV_dense.py: VI_SSM for the stochastic-volatility model and its
module-level driver (implementation: viforssms_amd/sv.py).  `python SV_dense.py --help`."""
import numpy as np

from viforssms_amd.sv import VI_SSM, make_theta_spec, run  # noqa: F401

np.random.seed(1)

if __name__ == "__main__":
    run()
