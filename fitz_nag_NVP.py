"""Drop-in for the reference's fitz_nag_NVP.py: VI_SSM for the FitzHugh-Nagumo model and its
module-level driver (implementation: viforssms_amd/fhn.py).  `python fitz_nag_NVP.py --help`."""
import numpy as np

from viforssms_amd.fhn import VI_SSM, make_theta_spec, run  # noqa: F401

np.random.seed(1)

if __name__ == "__main__":
    run()
