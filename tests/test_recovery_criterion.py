"""tests/recovery_util.py's posterior-recovery criterion on synthetic trajectories and on the float64 oracle's own
recovery run (profiles/r06/recovery/oracle_f64_seed1.log, committed): no GPU work."""
import json
import os

import glob

from tests.recovery_util import RECOVERY_BY, RECOVERY_EVERY, RECOVERY_SPAN, first_in_band, in_band, longest_band_run

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOOD = {"mean": [5.0, 0.5, 3.0], "sd": [0.3, 0.02, 0.05]}
OFF = {"mean": [7.0, 0.3, 3.2], "sd": [1.4, 0.14, 0.2]}
WIDE = {"mean": [5.0, 0.5, 3.0], "sd": [0.6, 0.02, 0.05]}


def test_band_run_criterion():
    """A run that holds the band for five checkpoints passes wherever it later goes; one that only touches it does
    not; a concentrated posterior off the generating values and a wide one at them are both outside."""
    assert in_band(GOOD) and not in_band(OFF) and not in_band(WIDE)
    assert longest_band_run([OFF, GOOD, GOOD, GOOD, GOOD, GOOD, OFF, OFF]) == 5
    assert first_in_band([{"step": 250, **OFF}, {"step": 500, **GOOD}]) == 500 and first_in_band([OFF]) is None
    assert longest_band_run([GOOD, WIDE, GOOD, GOOD, OFF, GOOD, GOOD]) == 2
    assert longest_band_run([]) == 0


def test_float64_oracle_run_meets_the_criterion():
    """The reference's algorithm in float64 (scripts/oracle_recovery.py, one 10,000-step run) reaches the posterior
    and holds it for the criterion's span, then leaves it: the criterion is met, and the final checkpoint is outside
    the band -- the departure the GPU runs show is the schedule's own."""
    recs = [json.loads(l) for l in open(os.path.join(ROOT, "profiles", "r06", "recovery", "oracle_f64_seed1.log"))
            if l.startswith('{"step"')]
    assert [r["step"] for r in recs][:2] == [RECOVERY_EVERY, 2 * RECOVERY_EVERY] and recs[-1]["step"] == 10000
    assert longest_band_run(recs) >= RECOVERY_SPAN and first_in_band(recs) <= RECOVERY_BY
    assert not in_band(recs[-1])


def test_gpu_seed_runs_meet_the_criterion():
    """The committed fp32 GPU runs (profiles/r06/recovery/gpu_seeds: four seeds x the library-GEMM theta branch, its
    reassociated variant and the HIP kernels, 10,000 steps each) all meet the criterion, while five of the twelve end
    outside the band: a last-step criterion would fail every form on some seed."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r06", "recovery", "gpu_seeds", "*_s[0-9].log")))
    assert len(files) == 12
    ends_out = 0
    for f in files:
        recs = [json.loads(l) for l in open(f) if l.startswith('{"step"')]
        assert recs[-1]["step"] == 10000
        assert longest_band_run(recs) >= RECOVERY_SPAN and first_in_band(recs) <= RECOVERY_BY, f
        ends_out += not in_band(recs[-1])
    assert ends_out == 5
