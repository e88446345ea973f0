"""bench.py's N-rank entry point on the CPU: ``python bench.py --gpus N`` without torchrun
spawns N ranks itself (gloo rendezvous on 127.0.0.1), a torchrun world that disagrees with
``--gpus`` fails loudly, and a real run asks for N GPUs before it starts anything."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "HIPZAP_SHARE_GPU")}
    env.update(kw)
    return env


def _json_lines(out: str):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def test_self_launch_spawns_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-check"], capture_output=True,
                       text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # only rank 0 reports
    assert lines[0]["n_gpus"] == 3 and lines[0]["ranks_seen"] == 3 and lines[0]["self_launched"]
    # the launcher spawned its ranks without mapping the HIP runtime (it never imports torch)
    assert lines[0]["launcher_hip_mapped"] == "0"


def test_launcher_path_imports_no_torch():
    """bench.py's N-rank launcher decision and GPU count run before (and without) ``import torch``:
    torch maps libamdhip64, and the launcher must not hold the HIP runtime while its ranks run."""
    code = ("import sys, runpy; sys.argv = ['bench.py', '--gpus', '2']; import bench, os; "
            "from hipzap.utils.gpucount import hip_mapped, visible_gpu_count; "
            "bench.check_gpus.__globals__; print('torch' in sys.modules, hip_mapped())")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT,
                       env=_env())
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["False", "False"]


def test_torchrun_world_mismatch_fails_loudly():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], capture_output=True,
                       text=True, timeout=120, cwd=ROOT,
                       env=_env(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "--gpus 2" in r.stderr and "WORLD_SIZE" in r.stderr


def test_missing_gpus_fail_before_spawning():
    # no GPU in this container: a real 2-GPU run must refuse instead of running one replica
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], capture_output=True, text=True,
                       timeout=120, env=_env(), cwd=ROOT)
    assert r.returncode != 0
    assert "needs 2 GPUs" in r.stderr and not _json_lines(r.stdout)
