"""Drop-in for the reference's lotka_volterra_partial.py: VI_SSM for the Lotka-Volterra model and its
module-level driver (implementation: viforssms_amd/lv.py).  `python lotka_volterra_partial.py --help`."""
import numpy as np

from viforssms_amd.lv import VI_SSM, make_theta_spec, run  # noqa: F401

np.random.seed(1)

if __name__ == "__main__":
    run()
