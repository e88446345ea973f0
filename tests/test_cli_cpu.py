"""CLI, settings, artifact store and packed-weight files (CPU)."""
import json
import os

import torch

from hipzap.__main__ import main
from hipzap.engine.packfile import load_packed, save_packed
from hipzap.models import registry
from hipzap.serve.artifacts import ArtifactStore
from hipzap.serve.settings import apply_environment, load_settings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_settings_template_and_env(tmp_path):
    cfg = json.load(open(os.path.join(ROOT, "zappa_settings.rename.json")))
    assert cfg["dev"]["app_function"] == "main.app"
    env = {}
    apply_environment(cfg, "dev", env)
    assert env["models_bucket"] == "models-bucket-name"
    p = tmp_path / "zs.json"
    p.write_text(json.dumps(cfg))
    env2 = {"HIPZAP_PORT": "9999"}
    st = load_settings(str(p), "dev", env2)
    assert st.models_bucket == "models-bucket-name" and st.port == 9999
    assert st.models["vit-b16"].name == "vit-b16-fp8" and st.models["resnet50"].contexts == 8
    assert st.lm_model_key == "models/rjokes/rjokes.model.pth"


def test_artifact_store_atomic_cache(tmp_path):
    bucket = tmp_path / "bucket"
    (bucket / "models" / "m").mkdir(parents=True)
    (bucket / "models" / "m" / "m.model.pth").write_bytes(b"abc")
    store = ArtifactStore(f"file://{bucket}", str(tmp_path / "cache"))
    p = store.fetch("models/m/m.model.pth")  # parent dirs created (main.py:33 bug fixed)
    assert open(p, "rb").read() == b"abc"
    (bucket / "models" / "m" / "m.model.pth").write_bytes(b"zzz")
    assert open(store.fetch("models/m/m.model.pth"), "rb").read() == b"abc"  # cached
    assert not [f for f in os.listdir(os.path.dirname(p)) if f.startswith(".part-")]


def test_upload_dir_local(tmp_path):
    src = tmp_path / "models" / "x"
    src.mkdir(parents=True)
    (src / "x.model.pth").write_bytes(b"1")
    bucket = tmp_path / "b"
    bucket.mkdir()
    copied = ArtifactStore(str(bucket)).upload_dir(str(tmp_path / "models"))
    assert copied == ["x/x.model.pth"] and (bucket / "models" / "x" / "x.model.pth").exists()


def test_packfile_roundtrip(tmp_path):
    a = registry.get("resnet18")
    params, cfg = a.pack(a.make_model().state_dict(), "cpu")
    path = str(tmp_path / "r18.hzpack")
    save_packed(params, cfg, path, "deadbeef")
    back, cfg2 = load_packed(path)
    assert cfg2 == cfg and set(back) == set(params)
    assert torch.equal(back["fc"].wf, params["fc"].wf) and back["fc"].cout == 1000


def test_packed_cache_validity(tmp_path):
    """<ckpt>.hzpack is used only if it was packed for this model from this exact file."""
    import os
    from hipzap.engine.packfile import find_packed, packed_path, source_stamp
    a = registry.get("resnet18")
    ck = str(tmp_path / "r.pth")
    torch.save(a.make_model().state_dict(), ck)
    assert find_packed(ck, "resnet18") is None
    params, cfg = a.pack(torch.load(ck, weights_only=True), "cpu")
    save_packed(params, cfg, packed_path(ck), model="resnet18", stamp=source_stamp(ck))
    assert find_packed(ck, "resnet18") == packed_path(ck)
    assert find_packed(ck, "resnet50") is None  # packed for another model
    st = os.stat(ck)
    os.utime(ck, ns=(st.st_atime_ns, st.st_mtime_ns + 10**9))  # checkpoint replaced
    assert find_packed(ck, "resnet18") is None
    open(packed_path(ck), "wb").write(b"garbage")  # partial/corrupt cache: ignored, not fatal
    assert find_packed(ck, "resnet18") is None


def test_cpu_backend_loads_checkpoint_path(tmp_path):
    from hipzap.serve.server import VisionBackend
    from hipzap.serve.settings import ModelSpec
    a = registry.get("resnet18")
    torch.manual_seed(0)
    m = a.make_model().eval()
    ck = str(tmp_path / "r.pth")
    torch.save(m.state_dict(), ck)
    be = VisionBackend("resnet18", ck, "cpu", "cpu", ModelSpec("resnet18"), False)
    x = torch.randn(1, 3, 32, 32)
    with torch.no_grad():
        assert torch.allclose(be(x), m(x))


def test_cli_pack_and_info(tmp_path, capsys):
    a = registry.get("resnet18")
    ck = tmp_path / "r.pth"
    torch.save(a.make_model().state_dict(), ck)
    main(["pack", "--model", "resnet18", "--ckpt", str(ck), "--out", str(tmp_path / "r.hzpack")])
    out = json.loads(capsys.readouterr().out)
    assert out["entries"] > 10
    main(["info"])
    assert "resnet50" in capsys.readouterr().out


def test_watchdog_and_fault_injection(monkeypatch):
    import pytest as _pt

    from hipzap.serve.server import RoundRobin
    from hipzap.utils.watchdog import DeviceWatchdog, InjectedFault, maybe_fault
    state = {"a": True, "b": False}
    wd = DeviceWatchdog(["a", "b"], timeout_s=0.05, probe=lambda d: (lambda: state[d]))
    assert wd.check_once() == {"a": True, "b": False} and wd.healthy_devices() == ["a"]

    class B:
        backend, cold_ms = "gpu", 1.0

        def __init__(self, tag):
            self.tag = tag

        def __call__(self):
            return self.tag
    rr = RoundRobin([B("a"), B("b")], ["a", "b"], lambda d: wd.healthy[d])
    assert [rr() for _ in range(4)] == ["a"] * 4  # unhealthy replica skipped
    monkeypatch.setenv("HIPZAP_FAULT", "load,rank3")
    with _pt.raises(InjectedFault):
        maybe_fault("rank3")
    maybe_fault("infer")


def test_tracing_ranges():
    from hipzap.utils.tracing import PhaseTimer, trace_range
    t = PhaseTimer()
    with trace_range("a", t):
        pass
    with trace_range("b", t):
        pass
    assert set(t.phases) == {"a", "b"} and "a=" in t.header()


def test_native_library_links():
    """libhipzap.so must dlopen with every symbol resolved (no GPU needed): catches kernels whose
    host stubs were silently not emitted, before a GPU box sees it."""
    import ctypes
    from hipzap import _native as N
    lib = N.lib()
    for sym in ("hz_conv_launch", "hz_conv2_launch", "hz_gemm_lds_launch", "hz_launch_kernel", "hz_prog_add_kernel",
                "hz_gemm_fp8_launch", "hz_softmax_launch", "hz_pool_fc_launch"):
        assert isinstance(getattr(lib, sym), ctypes._CFuncPtr)


def test_gpu_metrics_from_sysfs(tmp_path):
    """Per-GPU utilisation scraped from amdgpu sysfs files (a fake tree here)."""
    from hipzap.utils import gpu_metrics
    for i, busy in enumerate((37, 0)):
        dev = tmp_path / f"card{i}" / "device"
        (dev / "hwmon" / "hwmon3").mkdir(parents=True)
        (dev / "gpu_busy_percent").write_text(f"{busy}\n")
        (dev / "mem_info_vram_used").write_text("1073741824\n")
        (dev / "mem_info_vram_total").write_text("309237645312\n")
        (dev / "hwmon" / "hwmon3" / "power1_average").write_text("650000000\n")
    (tmp_path / "card0-DP-1").mkdir()  # a connector: ignored
    text = gpu_metrics.render(str(tmp_path))
    assert 'hipzap_gpu_busy_percent{gpu="0"} 37' in text and 'hipzap_gpu_busy_percent{gpu="1"} 0' in text
    assert 'hipzap_gpu_power_watts{gpu="0"} 650' in text
    assert gpu_metrics.render(str(tmp_path / "none")) == ""


def test_load_tuning_falls_back_to_highest_lower_concurrency(tmp_path, monkeypatch):
    """the conv table chosen for N streams is the one tuned for the highest
    concurrency <= N (c24 for 32 streams), else the latency table."""
    import json
    from hipzap.engine import engine as eng_mod
    from hipzap.engine import tune
    for suffix, tag in (("", "base"), ("_c8", "c8"), ("_c24", "c24")):
        (tmp_path / f"resnet50_bs1{suffix}.json").write_text(json.dumps({"tag": tag}))

    def table_path(model, batch, c=1):
        return tmp_path / (f"{model}_bs{batch}" + (f"_c{c}" if c > 1 else "") + ".json")
    monkeypatch.setattr(tune, "table_path", table_path)
    pick = lambda n: (eng_mod.load_tuning("resnet50", 1, n) or {}).get("tag")  # noqa: E731
    assert pick(32) == "c24" and pick(24) == "c24" and pick(16) == "c8" and pick(8) == "c8"
    assert pick(4) == "base" and pick(1) == "base"
    assert eng_mod.load_tuning("resnet50", 7, 4) is None
