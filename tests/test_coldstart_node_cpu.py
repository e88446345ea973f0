"""Node-level cold start launcher (hipzap/coldstart.py measure_node; VERDICT r3 "next round" 3a) on
the CPU: N fresh worker processes spawned together meet in the file rendezvous, and the figure is
timed from the launcher to the LAST rank; a failing rank fails the measurement instead of being
dropped from it. (``--dry``: the launcher and rendezvous only; the GPU workers run the same
plumbing plus RCCL init, the C1 weight broadcast and the first request.)"""
import pytest

from hipzap.coldstart import measure_node


@pytest.mark.parametrize("world", [1, 3])
def test_node_cold_start_launcher(world):
    r = measure_node("/nonexistent.hzplan", world, trials=3, dry=True, timeout=120)
    assert r["world"] == world and r["trials"] == 3 and len(r["all_ms"]) == 3
    assert r["min_ms"] <= r["p50_ms"] <= r["max_ms"] and r["p50_ms"] > 0
    assert r["torch_imported"] is False and 0 <= r["slowest_rank"] < world


def test_node_cold_start_fails_loudly_on_a_bad_rank():
    # not dry: every worker tries to open a plan that does not exist
    with pytest.raises(RuntimeError, match="node cold start"):
        measure_node("/nonexistent.hzplan", 2, trials=1, dry=False, timeout=120)


def test_a_dead_worker_stops_the_launch_at_once():
    """A worker that exits early leaves the others waiting in the rendezvous: the launcher stops
    the launch when it sees the exit, not at its timeout (on a real node: a rank whose device is
    not visible)."""
    import os
    import time
    t = time.time()
    with pytest.raises(RuntimeError, match="rank 1 exited 3"):
        measure_node("/nonexistent.hzplan", 3, trials=1, dry=True, timeout=120,
                     env=dict(os.environ, HIPZAP_COLD_FAIL_RANK="1"))
    assert time.time() - t < 30
