"""Generates tests/golden/ref_rng_replay.npz by IMPORTING THE REFERENCE's AR_dat_gen.py
(/root/reference, numpy only) and replaying the reference main.py's numpy-RNG call order:
  seed(1) at AR_dat_gen import, seed(1) at AR import (AR.py:18), data_gen(...) (AR_dat_gen.py:6-43),
  4 x np.random.permutation(arange(3)) (AR.py:383-385), np.random.choice(arange(0,T,M), p) per step
  (AR.py:263-265).
Run in the development container only (the reference does not exist on the GPU box); the output is
a data fixture (inputs/outputs), not reference source."""
import os
import sys
import tempfile

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_rng_replay.npz")


def main():
    sys.path.insert(0, REF)
    import AR_dat_gen  # noqa: E402  (the reference module)
    with tempfile.TemporaryDirectory() as d:
        np.random.seed(1)
        np.random.seed(1)
        AR_dat_gen.data_gen(5000, 1, 10.0, np.array([5.0, 0.5, 3.0]), 1.0, dat_dir=d)
        files = {n: np.loadtxt(os.path.join(d, "dat", n + ".txt"))
                 for n in ("AR_obs_partial", "AR_obs_binary", "AR_time_till")}
        perms = np.stack([np.random.permutation(np.arange(0, 3)) for _ in range(4)])
        T, M, p = 5000, 50, 50
        picks = np.stack([np.random.choice(np.arange(0, T, M), size=p, replace=(M * p >= T)) for _ in range(3)])
        # a second replay with impute=5 (the bench config's data)
        np.random.seed(1)
        np.random.seed(1)
        AR_dat_gen.data_gen(5000, 5, 10.0, np.array([5.0, 0.5, 3.0]), 1.0, dat_dir=d)
        imp5 = {n + "_imp5": np.loadtxt(os.path.join(d, "dat", n + ".txt"))
                for n in ("AR_obs_partial", "AR_obs_binary", "AR_time_till")}
    np.savez_compressed(OUT, perms=perms, picks=picks, **files, **imp5)
    print("wrote", OUT, {k: v.shape for k, v in {**files, **imp5}.items()}, perms.tolist(), picks[0][:8])


if __name__ == "__main__":
    main()
