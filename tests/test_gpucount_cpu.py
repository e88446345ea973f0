"""GPU discovery without HIP (hipzap/utils/gpucount.py): KFD topology nodes in sysfs, narrowed by
the visibility variables; what bench.py's launcher uses before spawning its ranks."""
import os
import subprocess
import sys

from hipzap.utils import gpucount as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _topology(tmp_path, simd_counts):
    root = tmp_path / "nodes"
    for i, s in enumerate(simd_counts):
        d = root / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {s}\ngfx_target_version 90500\n"
                                      f"unique_id {1000 + i}\ndrm_render_minor {128 + i}\n")
    return str(root)


def test_counts_gpu_nodes_only(tmp_path):
    root = _topology(tmp_path, [0, 1024, 1024, 1024, 1024, 1024, 1024, 1024, 1024])  # a CPU node + 8 GPUs
    assert len(G.kfd_gpu_nodes(root)) == 8
    assert G.visible_gpu_count({}, root) == 8
    assert [n["node"] for n in G.kfd_gpu_nodes(root)] == [str(i) for i in range(1, 9)]


def test_visibility_variables_narrow_the_count(tmp_path):
    root = _topology(tmp_path, [0] + [1024] * 8)
    assert G.visible_gpu_count({"ROCR_VISIBLE_DEVICES": "3"}, root) == 1
    assert G.visible_gpu_count({"HIP_VISIBLE_DEVICES": "0,1,2,3"}, root) == 4
    assert G.visible_gpu_count({"CUDA_VISIBLE_DEVICES": "0,1", "HIP_VISIBLE_DEVICES": "0,1,2"}, root) == 2
    assert G.visible_gpu_count({"HIP_VISIBLE_DEVICES": ""}, root) == 8  # (unset in effect)
    env = G.environment({"HIP_VISIBLE_DEVICES": "5"}, root)
    assert env["visibility_vars"] == {"HIP_VISIBLE_DEVICES": "5"} and env["kfd_gpu_nodes"] == 8
    assert env["kfd_nodes"] == 9 and env["visible_gpus"] == 1


def test_no_topology_means_no_gpus(tmp_path):
    assert G.visible_gpu_count({}, str(tmp_path / "absent")) == 0


def test_discovery_never_maps_hip():
    code = ("from hipzap.utils import gpucount as G; n = G.visible_gpu_count(); "
            "print(n, G.hip_mapped())")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split()[1] == "False"
