"""Cold-start children see only their own GPU (hipzap/coldstart.py isolated_env)."""
from hipzap.coldstart import isolated_env


def test_isolates_to_one_physical_gpu():
    env, dev = isolated_env({"PATH": "/bin"}, 5)
    assert env["ROCR_VISIBLE_DEVICES"] == "5" and dev == 0 and env["PATH"] == "/bin"


def test_respects_launcher_visibility_and_opt_out():
    env = {"ROCR_VISIBLE_DEVICES": "3"}  # already one ROCr agent: left alone
    assert isolated_env(env, 0) == (env, 0)
    env = {"ROCR_VISIBLE_DEVICES": "3", "HIP_VISIBLE_DEVICES": "0"}  # (the serving lease's pair)
    assert isolated_env(env, 0) == (env, 0)
    env = {"HIPZAP_COLD_ISOLATE": "0"}
    assert isolated_env(env, 4) == (env, 4)
    for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):  # round-5 behaviour on request
        env = {k: "2,3", "HIPZAP_COLD_NARROW": "0"}
        assert isolated_env(env, 1) == (env, 1)


def test_a_hip_level_list_is_narrowed_at_the_rocr_level():
    """A launcher that sets only HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES leaves ROCr opening
    every agent it can see; the one-GPU child gets ROCR_VISIBLE_DEVICES=<physical index> and
    HIP_VISIBLE_DEVICES=0 (VERDICT r5 next #2c)."""
    from hipzap.coldstart import narrow_env
    for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL"):
        env, dev = isolated_env({k: "2,3", "PATH": "/bin"}, 1)
        assert dev == 0 and env["ROCR_VISIBLE_DEVICES"] == "3" and env["HIP_VISIBLE_DEVICES"] == "0"
        assert env["PATH"] == "/bin" and (k == "HIP_VISIBLE_DEVICES" or k not in env)
    assert narrow_env({"HIP_VISIBLE_DEVICES": "4"}, 0)[2] == "rocr_from_hip_visible_devices"
    assert narrow_env({}, 2)[:2] == ({"ROCR_VISIBLE_DEVICES": "2"}, 0)
    # a multi-GPU ROCr list (an 8-GPU node's launcher): narrowed to the rank's entry
    env, dev = isolated_env({"ROCR_VISIBLE_DEVICES": "0,1,2,3,4,5,6,7"}, 5)
    assert env == {"ROCR_VISIBLE_DEVICES": "5"} and dev == 0
    env, dev = isolated_env({"ROCR_VISIBLE_DEVICES": "4,5,6,7", "HIP_VISIBLE_DEVICES": "3,2"}, 1)
    assert env == {"ROCR_VISIBLE_DEVICES": "6", "HIP_VISIBLE_DEVICES": "0"} and dev == 0
    assert narrow_env({"ROCR_VISIBLE_DEVICES": "GPU-a,GPU-b"}, 1)[:2] == ({"ROCR_VISIBLE_DEVICES": "GPU-b"}, 0)
    assert narrow_env({"ROCR_VISIBLE_DEVICES": "0,1"}, 1)[2] == "rocr_from_rocr_visible_devices"
    # an index the list does not have, a UUID entry, or two disagreeing lists: unchanged
    for env, d in (({"HIP_VISIBLE_DEVICES": "0"}, 3), ({"HIP_VISIBLE_DEVICES": "GPU-abc"}, 0),
                   ({"HIP_VISIBLE_DEVICES": "1", "CUDA_VISIBLE_DEVICES": "0"}, 0)):
        assert narrow_env(env, d) == (env, d, "unchanged")


def test_interleaved_cold_start_alternates_and_drops_failed_routes(monkeypatch):
    """bench.py measures the torch-free routes (plan, .pth-lite, native) in alternation: trial k of
    every route before trial k + 1 of any, so box drift lands on all alike; a route whose child
    fails drops out with its error and the others finish."""
    from hipzap import coldstart as cs
    calls = []
    monkeypatch.setattr(cs, "_fresh_cmd", lambda mode, path, model, device, extra: [mode])

    def trial(cmd, mode, env, timeout):
        calls.append(mode)
        if mode == "native" and calls.count("native") == 2:
            raise RuntimeError("child failed")
        return 100.0 + len(calls), {"phases_ms": {"hip_init_ms": 1.0}}

    monkeypatch.setattr(cs, "_fresh_trial", trial)
    out = cs.measure_fresh_interleaved({"plan": ("plan", "p", "resnet50", None),
                                        "pth_lite": ("pth-lite", "c", "resnet50", None),
                                        "native": ("native", "p", "resnet50", None)}, trials=3, env={})
    assert calls == ["plan", "pth-lite", "native", "plan", "pth-lite", "native", "plan", "pth-lite"]
    assert out["plan"]["trials"] == 3 and out["pth_lite"]["trials"] == 3
    assert out["plan"]["all_ms"] == [101.0, 104.0, 107.0] and out["plan"]["p50_ms"] == 104.0
    assert "error" in out["native"] and out["plan"]["interleaved_with"] == ["native", "pth_lite"]


def test_child_argv_parser():
    """The cold-start child parses its argv by hand (no argparse in the measured window)."""
    import pytest
    from hipzap import coldstart as cs
    a = cs._parse(["node", "x.hzplan", "--rank", "1", "--world=2", "--rdzv", "/tmp/r", "--dry"])
    assert (a.mode, a.path, a.rank, a.world, a.rdzv, a.dry, a.device, a.model) == \
        ("node", "x.hzplan", 1, 2, "/tmp/r", True, 0, "resnet50")
    a = cs._parse(["lm", "ck.pth", "--vocab", "itos.pkl", "--words", "20", "--device", "3"])
    assert (a.mode, a.vocab, a.words, a.device, a.dry) == ("lm", "itos.pkl", 20, 3, False)
    a = cs._parse(["plan", "a=b.hzplan"])  # '=' in a positional is a path, not an option
    assert a.path == "a=b.hzplan"
    for bad in (["plan"], ["bogus", "p"], ["plan", "p", "--nope"], ["plan", "p", "--rank"], ["plan", "p", "q"]):
        with pytest.raises(SystemExit):
            cs._parse(bad)


def test_trial_gap_default_and_override(monkeypatch):
    """Each fresh cold-start child starts on an idle GPU by default (300 ms after the previous one
    exited); HIPZAP_COLD_GAP_MS=0 gives the back-to-back trials; a per-call gap wins over both."""
    from hipzap import coldstart
    monkeypatch.delenv("HIPZAP_COLD_GAP_MS", raising=False)
    assert coldstart.trial_gap_s() == 0.3
    monkeypatch.setenv("HIPZAP_COLD_GAP_MS", "0")
    assert coldstart.trial_gap_s() == 0.0
    slept = []
    monkeypatch.setattr(coldstart.time, "sleep", slept.append)

    class R:
        returncode, stderr = 0, ""
        stdout = '{"t_first": 1e12, "phases_ms": {}}\n'
    import subprocess
    monkeypatch.setattr(subprocess, "run", lambda *a, **k: R())
    coldstart._fresh_trial(["x"], "plan", None, 1.0, 0.05)
    coldstart._fresh_trial(["x"], "plan", None, 1.0)
    assert slept == [0.05]
