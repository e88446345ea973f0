#!/usr/bin/env python3
"""AWD-LSTM decode step time against the vocabulary size (the decoder's weight stream), batched
engine (engine/lmbatch.py), reference dimensions otherwise (emb 1000, hidden 1150, 3 layers).

A lone 200-word request per vocabulary size gives µs per step; the step is the three layer launches
(independent of V) plus the decoder, whose bytes grow with V (Vp x 1024 bf16 + the W_hh rows it
also computes). A fit step(V) = a + V * 2048 B / rate gives the decoder's effective stream rate;
a rate that drops as V grows past the point where the step's working set leaves the 256 MiB
Infinity Cache would show the decoder is cache-capacity-bound rather than at its HBM rate.
Prints one JSON line per V and a summary line."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from hipzap.engine.lmbatch import LMBatchEngine, pack_lmb
    from hipzap.models.awd_lstm import reference_lm
    vocabs = [int(v) for v in (sys.argv[1:] or ["8000", "20000", "40000", "60000", "90000"])]
    rows = []
    for V in vocabs:
        torch.manual_seed(0)
        sd = reference_lm(V).eval().state_dict()
        eng = LMBatchEngine(pack_lmb(sd, "cuda:0"), "cuda:0", rows=32, unroll=8, exclude_ids=[2, 5, 6])
        eng.run_tokens([0], 200, 1)
        ts = []
        for i in range(7):
            t = time.perf_counter()
            eng.run_tokens([0], 200, 3 + i)
            ts.append((time.perf_counter() - t) * 1e3)
        ms = statistics.median(ts)
        r = {"V": V, "lone_request_ms": round(ms, 3), "us_per_step": round(ms * 1e3 / 201, 2),
             "decoder_MB": round(V * 1024 * 2 / 1e6, 1)}
        rows.append(r)
        print(json.dumps(r), flush=True)
        eng.close()
        del eng, sd
        torch.cuda.empty_cache()
    if len(rows) >= 2:
        slopes = [((b["us_per_step"] - a["us_per_step"]) / (b["V"] - a["V"]), a["V"], b["V"])
                  for a, b in zip(rows, rows[1:])]
        print(json.dumps({"marginal_decoder_TB_s": [
            {"V": f"{lo}-{hi}", "TB_s": round(2048 / max(s * 1e6, 1e-9) / 1e6 * 1e6, 2)} for s, lo, hi in slopes]}))


if __name__ == "__main__":
    main()
