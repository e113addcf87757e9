"""Drop-in for the reference's AR_dat_gen.py: ``data_gen(T, impute, x0, theta, obs_std, dat_dir)``
(implementation: viforssms_amd/data.py).  Importing it seeds the global numpy RNG with 1, as the
reference module does."""
import numpy as np

from viforssms_amd.data import data_gen  # noqa: F401

np.random.seed(1)

if __name__ == "__main__":
    data_gen(T=5000, impute=1, x0=10.0, theta=np.array([5.0, .5, 3.0]), obs_std=1.)
