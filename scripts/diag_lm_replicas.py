#!/usr/bin/env python3
"""GET /inference throughput with R batched AWD-LSTM engines sharing one packed weight set (each
its own 32 request rows, scheduler and stream): does a second engine's decode step overlap the
first's on the chip? Clients pick engines round-robin. Reference dims, V = 60000, random-init,
200 words per request; prints one JSON line per (replicas, stream kind, clients).

    python scripts/diag_lm_replicas.py [--clients 32,64,128] [--requests 6]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def _arg(name, default):
    return sys.argv[sys.argv.index(name) + 1] if name in sys.argv else default


def main():
    import torch
    from bench_lm_batch import run_load
    from hipzap.engine.lmbatch import LMBatchEngine, pack_lmb
    from hipzap.models.awd_lstm import reference_lm
    clients = [int(c) for c in _arg("--clients", "32,64,128").split(",")]
    requests = int(_arg("--requests", "6"))
    torch.manual_seed(0)
    packed = pack_lmb(reference_lm(60000).eval().state_dict(), "cuda:0")
    for reps, hiprio in ((2, True), (1, False), (2, False)):
        engines = []
        for i in range(reps):  # hiprio: the second engine's stream at high priority (a queue set of its own)
            engines.append(LMBatchEngine(packed, "cuda:0", rows=32, exclude_ids=[2, 5, 6],
                                         priority=-1 if hiprio and i else 0))
        for e in engines:
            e.run_tokens([0], 200, 1)
        ctr = [0]

        def fn(ids, words, seed):
            ctr[0] += 1
            return engines[ctr[0] % reps].run_tokens(ids, words, seed)
        for c in clients:
            r = run_load(fn, c, requests, 200)
            print(json.dumps({"replicas": reps, "hiprio": hiprio, **r}), flush=True)
        for e in engines:
            e.close()
        del engines
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
