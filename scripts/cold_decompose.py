#!/usr/bin/env python3
"""Decompose the cold-start floor: the environment a fresh one-GPU worker
starts in (visibility variables, KFD topology nodes, render nodes) and, over >= --trials fresh
processes per arm, interleaved, where HIP init's time goes (scripts/native/hsa_init_probe.cpp):
hsa_init / agent + pool enumeration / first AQL queue / HIP's own increment / first stream.

Arms: ``hip`` (HIP alone, the plain floor) and ``hsa`` (the ROCr phases first, then HIP on the
live runtime), each in the environment as given and narrowed to one ROCr agent
(ROCR_VISIBLE_DEVICES=<k> + HIP_VISIBLE_DEVICES=0, k = the physical index HIP would use).
Writes one JSON file; prints a summary."""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hipzap.utils.gpucount import environment  # noqa: E402

PROBE = os.path.join(ROOT, "scripts", "native", "hsa_init_probe")


def narrowed(env: dict, device: int = 0) -> dict:
    from hipzap.coldstart import narrow_env
    return narrow_env(env, device)[0]


def main():
    trials = int(sys.argv[sys.argv.index("--trials") + 1]) if "--trials" in sys.argv else 12
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else "gpurun_out/cold_decompose.json"
    base = dict(os.environ)
    arms = {"hip": ([PROBE, "--hip-only"], base), "hsa": ([PROBE], base), "null_first": ([PROBE, "--null-first"], base),
            "hip_narrow": ([PROBE, "--hip-only"], narrowed(base)), "hsa_narrow": ([PROBE], narrowed(base))}
    res = {"environment": environment(base),
           "env_vars": {k: v for k, v in base.items() if any(s in k for s in ("VISIBLE", "ROCR", "HSA_", "HIP_", "GPU_"))},
           "narrowed_vars": {k: v for k, v in narrowed(base).items() if "VISIBLE" in k},
           "trials": trials, "arms": {a: [] for a in arms}}
    for t in range(trials):  # interleaved: box drift hits every arm alike
        for a, (cmd, env) in arms.items():
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=60, env=env)
            lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            res["arms"][a].append(json.loads(lines[-1]) if lines else {"error": r.stderr[-500:], "rc": r.returncode})
        print(f"trial {t + 1}/{trials}", flush=True)
    summ = {}
    for a, rows in res["arms"].items():
        ok = [r for r in rows if "total_ms" in r]
        summ[a] = {k: round(statistics.median(r[k] for r in ok), 2) for k in ok[0] if k not in
                   ("rc", "hip_only", "null_first", "agents", "gpu_agents", "pools", "hip_devices")} \
            if ok else {"error": rows[-1]}
        if ok and "gpu_agents" in ok[0]:
            summ[a].update(gpu_agents=ok[0]["gpu_agents"], agents=ok[0]["agents"], hip_devices=ok[0]["hip_devices"],
                           total_min=round(min(r["total_ms"] for r in ok), 2),
                           total_max=round(max(r["total_ms"] for r in ok), 2))
    res["median"] = summ
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({"environment": res["environment"], "env_vars": res["env_vars"], "median": summ}, indent=1))


if __name__ == "__main__":
    main()
