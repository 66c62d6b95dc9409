"""MI355X: bench.py's captured multi-step replay -- G training steps per hipGraph launch, each
with its own batch gather and update -- follows exactly the trajectory of one step per replay
(bit-identical final loss), across an epoch boundary too."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, diag=False):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--mlp-dims", "1024,512,512",
           "--dataset", "640", "--batch", "32", "--device-warmup-ms", "0", *args]
    if not diag:
        cmd.append("--no-diag")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])


def test_graph_steps_trajectory_is_bit_identical():
    # 20 steps per epoch: warm-up 3 + 30 timed steps cross an epoch boundary mid-group
    recs = {g: _bench("--steps", "30", "--warmup", "3", "--graph-steps", str(g))
            for g in (1, 4)}
    assert recs[1]["config"]["graph_steps"] == 1 and recs[4]["config"]["graph_steps"] == 4
    assert recs[1]["config"]["final_loss"] == recs[4]["config"]["final_loss"], recs


def test_rehearsal_diagnostic_replays_the_timed_form():
    """The one-GPU rehearsal of the W > 1 schedule (diagnostics) is captured and timed in the
    measured step's replay form -- G training steps per graph launch -- so rehearsal_over_dp1
    compares schedules, not graph-launch counts."""
    rec = _bench("--steps", "12", "--warmup", "2", diag=True)
    d = rec["diagnostics"]
    assert d["mode"] == "graph"
    assert d["rehearsal_graph_steps"] == rec["config"]["graph_steps"] == 4, d
    assert d["rehearsal_ms"] > 0 and d["rehearsal_schedule_ms"] > 0, d
    assert d["rehearsal_buckets"] >= 1, d
