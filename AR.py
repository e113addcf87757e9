"""Drop-in for the reference's AR.py: VI_SSM and main() for the AR(1) model
(implementation: viforssms_amd/ar.py).  Importing it seeds the global numpy RNG with 1 (AR.py:18)."""
import numpy as np

from viforssms_amd.ar import VI_SSM, build_theta_spec, main  # noqa: F401

np.random.seed(1)

if __name__ == "__main__":
    # paper defaults (AR.py:407-419)
    p = 50
    kernel_len = 50
    T = 5000.
    batch_dims = 50
    network_dims = [50] * 3
    no_flows = 3
    priors = [(0., 10.0)] * 3
    feat_window = 10
    x0 = 10.0
    obs_std = 1.0
    main(p, kernel_len, T, batch_dims, network_dims, no_flows, priors, feat_window, x0, obs_std)
