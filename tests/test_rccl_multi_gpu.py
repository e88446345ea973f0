"""RCCL at world >= 2 (VERDICT r3 "next round" 3b): skipped on a one-GPU box, runs as-is on a
multi-GPU node. Every rank is a FRESH process (hipzap/parallel/selftest.py), one per GPU:

* torch-free processes: C1 broadcast, C2 scatter, C3 gather bitwise and the C4 health all-reduce
  returning N, over the native communicator (csrc/comm/comm.cpp);
* torch-imported processes (bench.py's library mix): the same through the tensor interface, and
  DPExecutor over RCCL (ResNet-18 global batch scattered / run per shard / gathered) bitwise equal
  to rank 0 running every shard alone, including the one-host-sync asynchronous step, and
  DPPipeline with three steps in flight (the collectives in pipelined order);
* the node-level cold start (hipzap/coldstart.py measure_node): N torch-free plan workers, RCCL
  rendezvous, rank 0 broadcasts the weight blob, every rank serves a finite first request.
"""
import json
import os
import subprocess
import sys
import tempfile

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NDEV = torch.cuda.device_count()  # does not initialise HIP on this image
WORLD = NDEV  # the whole node (8 on an MI355X node): what the driver's scaling run will use
multi = pytest.mark.skipif(NDEV < 2, reason=f"needs >= 2 GPUs (this box has {NDEV})")


def _run_ranks(mode: str, world: int, timeout: float = 240.0) -> list:
    """One fresh process per rank; each rank's stdout / stderr go to its own file (a rank blocked
    on a full pipe while the test waits on another rank would deadlock the collective)."""
    import time
    rdzv = tempfile.mkdtemp(prefix="hz_selftest_")
    files = [(open(os.path.join(rdzv, f"r{r}.out"), "w+"), open(os.path.join(rdzv, f"r{r}.err"), "w+"))
             for r in range(world)]
    procs = [subprocess.Popen([sys.executable, "-m", "hipzap.parallel.selftest", "--mode", mode, "--rank", str(r),
                               "--world", str(world), "--rdzv", rdzv], cwd=ROOT, stdout=fo, stderr=fe, text=True)
             for r, (fo, fe) in enumerate(files)]
    outs = []
    try:
        deadline = time.time() + timeout
        for p in procs:  # every rank runs concurrently; wait for all within one deadline
            p.wait(timeout=max(1.0, deadline - time.time()))
        for r, (p, (fo, fe)) in enumerate(zip(procs, files)):
            fo.seek(0)
            fe.seek(0)
            so, se = fo.read(), fe.read()
            lines = [ln for ln in so.splitlines() if ln.startswith("{")]
            assert lines, f"rank {r} printed nothing (rc {p.returncode}): {se[-3000:]}"
            outs.append(json.loads(lines[-1]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        for fo, fe in files:
            fo.close()
            fe.close()
    return outs


@multi
def test_rccl_collectives_torch_free():
    outs = _run_ranks("lite", WORLD)
    for o in outs:
        assert o["ok"] and o["torch_imported"] is False, o
    assert outs[0]["checks"]["gather"] and all(o["checks"]["health"] for o in outs)


@multi
def test_rccl_collectives_and_dp_with_torch_loaded():
    outs = _run_ranks("torch", WORLD)
    for o in outs:
        assert o["ok"], o
    assert outs[0]["checks"]["dp_vs_shards_alone"] and outs[0]["checks"]["dp_async_equals_sync"]
    assert outs[0]["checks"]["dp_pipeline_vs_shards_alone"]


@multi
def test_node_cold_start_world(tmp_path):
    from hipzap.coldstart import measure_node
    from hipzap.engine.plan import export_from_checkpoint
    from hipzap.models.resnet import randomize_bn, resnet50
    torch.manual_seed(0)
    ck = str(tmp_path / "r50.pth")
    torch.save(randomize_bn(resnet50()).eval().state_dict(), ck)
    plan = export_from_checkpoint("resnet50", ck, str(tmp_path / "r50.hzplan"))
    r = measure_node(plan, WORLD, trials=2, timeout=240)
    assert r["world"] == WORLD and r["p50_ms"] > 0 and r["torch_imported"] is False


@pytest.mark.parametrize("mode", ["lite", "torch"])
def test_selftest_world1(mode):
    """The same worker at world 1 (runs on the one-GPU pool): the script's checks themselves."""
    outs = _run_ranks(mode, 1)
    assert outs[0]["ok"], outs[0]
