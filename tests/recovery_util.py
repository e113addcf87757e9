"""The posterior-recovery criterion of tests/test_gpu_posterior.py (CPU-importable; checked on synthetic
trajectories by tests/test_recovery_criterion.py).

The reference schedule (Adamax lr 1e-3, beta1 0.95, clip 2.5e8, p 50 windows of M 50; AR.py:226-234, 263-265,
optimisers/adamax.py:42-58) does not settle: the float64 oracle's own run of it (scripts/oracle_recovery.py,
profiles/r06/recovery/oracle_f64_seed1.log: the reference's algorithm in exact arithmetic, no product code) reaches
the posterior by step ~5,000, holds it to ~8,000 (sd(theta0) 0.33-0.36), then wanders off along the
theta0 / (1 - theta1) = 10 ridge (step 10,000: mean (7.1, 0.31, 3.2), sd 1.4).  When that departure starts depends on
the draws and on last-bit rounding, for every theta-branch form alike: over four seeds of the GPU's fp32 run
(profiles/r06/recovery/SUMMARY.md) every run of every form enters the band by step 3,500 and holds it for 3,500 to
7,250 steps, and 5 of the 12 runs have left it by step 10,000 (the library-GEMM form 1, its reassociated variant 2,
the HIP kernels 2).  So the criterion is that training REACHES the posterior: for every seed, the posterior mean lies
in the stated band and its sd below the stated bound by step RECOVERY_BY and over RECOVERY_SPAN consecutive
checkpoints RECOVERY_EVERY steps apart -- not where one trajectory happens to sit at its last step."""
from __future__ import annotations

# band for the posterior mean of (theta0, theta1, e^theta2) around the generating values (5, 0.5, 3)
# (AR_dat_gen.py:13-15; e^theta2 is the transition noise sd, AR.py:172-176), and the sd bound
RECOVERY_BAND = {"theta0": (5.0, 0.5), "theta1": (0.5, 0.05), "e^theta2": (3.0, 0.15)}
RECOVERY_SD_MAX = (0.5, 0.05, 0.15)
RECOVERY_EVERY = 250
RECOVERY_SPAN = 8                       # consecutive checkpoints: 2,000 steps in the band (shortest seen: 14)
RECOVERY_BY = 5000                      # the band is entered by this step (latest seen: 3,500)
RECOVERY_SEEDS = {"fp32": (1, 2, 3), "bf16": (1,)}   # Philox seeds of the eps / q(theta) base draws, each run once


def in_band(rec) -> bool:
    m, sd = rec["mean"], rec["sd"]
    return (all(abs(v - t) <= b for (t, b), v in zip(RECOVERY_BAND.values(), m))
            and all(v < smax for v, smax in zip(sd, RECOVERY_SD_MAX)))


def first_in_band(recs):
    """The step of the first checkpoint in the band (None: never)."""
    return next((r["step"] for r in recs if in_band(r)), None)


def longest_band_run(recs) -> int:
    """The longest run of consecutive checkpoints in the band."""
    best = cur = 0
    for r in recs:
        cur = cur + 1 if in_band(r) else 0
        best = max(best, cur)
    return best
