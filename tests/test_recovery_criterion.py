"""tests/recovery_util.py's posterior-recovery criterion on synthetic trajectories and on the float64 oracle's own
recovery run (profiles/r06/recovery/oracle_f64_seed1.log, committed): no GPU work."""
import json
import os

from tests.recovery_util import RECOVERY_EVERY, RECOVERY_SPAN, in_band, longest_band_run

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOOD = {"mean": [5.0, 0.5, 3.0], "sd": [0.3, 0.02, 0.05]}
OFF = {"mean": [7.0, 0.3, 3.2], "sd": [1.4, 0.14, 0.2]}
WIDE = {"mean": [5.0, 0.5, 3.0], "sd": [0.6, 0.02, 0.05]}


def test_band_run_criterion():
    """A run that holds the band for five checkpoints passes wherever it later goes; one that only touches it does
    not; a concentrated posterior off the generating values and a wide one at them are both outside."""
    assert in_band(GOOD) and not in_band(OFF) and not in_band(WIDE)
    assert longest_band_run([OFF, GOOD, GOOD, GOOD, GOOD, GOOD, OFF, OFF]) == 5
    assert longest_band_run([GOOD, WIDE, GOOD, GOOD, OFF, GOOD, GOOD]) == 2
    assert longest_band_run([]) == 0


def test_float64_oracle_run_meets_the_criterion():
    """The reference's algorithm in float64 (scripts/oracle_recovery.py, one 10,000-step run) reaches the posterior
    and holds it for the criterion's span, then leaves it: the criterion is met, and the final checkpoint is outside
    the band -- the departure the GPU runs show is the schedule's own."""
    recs = [json.loads(l) for l in open(os.path.join(ROOT, "profiles", "r06", "recovery", "oracle_f64_seed1.log"))
            if l.startswith('{"step"')]
    assert [r["step"] for r in recs][:2] == [RECOVERY_EVERY, 2 * RECOVERY_EVERY] and recs[-1]["step"] == 10000
    assert longest_band_run(recs) >= RECOVERY_SPAN
    assert not in_band(recs[-1])
