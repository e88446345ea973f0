"""Cold-start children see only their own GPU (hipzap/coldstart.py isolated_env)."""
from hipzap.coldstart import isolated_env


def test_isolates_to_one_physical_gpu():
    env, dev = isolated_env({"PATH": "/bin"}, 5)
    assert env["ROCR_VISIBLE_DEVICES"] == "5" and dev == 0 and env["PATH"] == "/bin"


def test_respects_launcher_visibility_and_opt_out():
    for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        env = {k: "2,3"}
        assert isolated_env(env, 1) == (env, 1)
    env = {"HIPZAP_COLD_ISOLATE": "0"}
    assert isolated_env(env, 4) == (env, 4)
