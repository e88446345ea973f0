"""GET /inference without torch (hipzap/lmlite.py) on MI355X: the engine built from the .pth by
the weights-only reader + raw upload + device packing samples the SAME tokens and logits as the
torch-built LMBatchEngine for fixed seeds (bitwise), honours the W_hh checkpoint quirk (SURVEY.md
§5.4: a zeroed ``_raw`` decoy is ignored), handles an untied decoder, and cold-starts in a fresh
process with torch never imported (VERDICT r3 "next round" 2)."""
import json
import os
import pickle
import subprocess
import sys

import pytest
import torch

from hipzap.engine.lmbatch import LMBatchEngine, pack_lmb
from hipzap.lmlite import LMLiteEngine
from hipzap.models.awd_lstm import reference_lm

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
V = 3000


@pytest.fixture(scope="module")
def ckpt(tmp_path_factory):
    d = tmp_path_factory.mktemp("lmlite")
    torch.manual_seed(11)
    sd = reference_lm(V).eval().state_dict()
    for l in range(3):  # decoy: the effective W_hh is module.weight_hh_l0
        sd[f"0.rnns.{l}.weight_hh_l0_raw"] = torch.zeros_like(sd[f"0.rnns.{l}.weight_hh_l0_raw"])
    p = str(d / "lm.pth")
    torch.save(sd, p)
    itos = ["xxunk", "xxpad", "xxup", "xxfld", "xxrep"] + [f"w{i}" for i in range(V - 5)]
    vocab = str(d / "lm.itos.pkl")
    with open(vocab, "wb") as f:
        pickle.dump(itos, f)
    return p, sd, vocab


def test_tokens_and_logits_bitwise_the_torch_engine(ckpt):
    p, sd, _ = ckpt
    ref = LMBatchEngine(pack_lmb(sd, "cuda:0"), "cuda:0", rows=16, unroll=4, exclude_ids=[2, 3, 4],
                        record_logits=True)
    lite = LMLiteEngine(p, rows=16, unroll=4, exclude_ids=[2, 3, 4], record_logits=True)
    try:
        for seed, prompt in ((1, [0]), (7, [5, 9, 11]), (123456789, [17] * 6)):
            ta, la = ref.run_tokens(prompt, 40, seed=seed, logits=True)
            tb, lb = lite.run_tokens(prompt, 40, seed=seed, logits=True)
            assert ta == tb, seed
            assert torch.equal(la, torch.frombuffer(bytearray(lb), dtype=torch.float32)), seed
    finally:
        ref.close()
        lite.close()


def test_whh_quirk_and_untied_decoder(ckpt, tmp_path):
    p, sd, _ = ckpt
    raw_sd = dict(sd)
    for l in range(3):
        raw_sd.pop(f"0.rnns.{l}.module.weight_hh_l0")  # a loader that took _raw (zeros) would compute this
    ref = LMBatchEngine(pack_lmb(sd, "cuda:0"), "cuda:0", rows=16, unroll=4, record_logits=True)
    raw = LMBatchEngine(pack_lmb(raw_sd, "cuda:0"), "cuda:0", rows=16, unroll=4, record_logits=True)
    lite = LMLiteEngine(p, rows=16, unroll=4, record_logits=True)
    try:
        # logits after a multi-token prompt (the recurrent term matters; sampled tokens of a
        # random-init model are decided by the Gumbel noise, not by the nearly flat logits)
        prompt = [5, 9, 11, 13]
        la = torch.frombuffer(bytearray(lite.run_tokens(prompt, 1, seed=3, logits=True)[1]), dtype=torch.float32)
        lr = raw.run_tokens(prompt, 1, seed=3, logits=True)[1]
        lm = ref.run_tokens(prompt, 1, seed=3, logits=True)[1]
        assert torch.equal(la, lm)  # the module weight, as the torch packer takes it
        assert (la - lr).abs().max().item() > 1e-3 * la.abs().max().item()  # not the zeroed _raw decoy
    finally:
        ref.close()
        raw.close()
        lite.close()
    # untied: a decoder weight in its own storage (different values) is packed separately
    un = dict(sd)
    un["1.decoder.weight"] = sd["0.encoder.weight"].clone() * 0.5
    q = str(tmp_path / "untied.pth")
    torch.save(un, q)
    ref = LMBatchEngine(pack_lmb(un, "cuda:0"), "cuda:0", rows=16, unroll=4)
    lite = LMLiteEngine(q, rows=16, unroll=4)
    try:
        assert lite.geo.dec_key == "1.decoder.weight"
        assert ref.run_tokens([4, 8], 30, seed=9) == lite.run_tokens([4, 8], 30, seed=9)
    finally:
        ref.close()
        lite.close()


def test_fresh_process_cold_start_is_torch_free(ckpt):
    p, _, vocab = ckpt
    out = subprocess.run([sys.executable, "-m", "hipzap.coldstart", "lm", p, "--vocab", vocab], cwd=ROOT,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert r["ok"] and r["torch_imported"] is False and r["numpy_imported"] is False and r["vocab"] == V


def test_lazy_capture_is_bitwise_the_eager_engine_under_load(ckpt):
    """capture="lazy": the lone first request replays the one-request graphs, the
    other programs run launch by launch until the background capture publishes them -- while 12
    concurrent requests run through them. Every request's tokens equal the eagerly captured
    engine's for the same seed, and afterwards every program is captured."""
    import threading
    from hipzap import _native as N
    p, _, _ = ckpt
    eager = LMLiteEngine(p, rows=32, unroll=4, exclude_ids=[2, 3, 4], capture=True)
    lazy = LMLiteEngine(p, rows=32, unroll=4, exclude_ids=[2, 3, 4], capture="lazy")
    try:
        core = lazy.core
        assert core._pending and all(N.lib().hz_prog_is_captured(q) for q in core.progs_solo)
        first = lazy.run_tokens([0], 30, seed=5)  # starts the deferred capture
        assert first == eager.run_tokens([0], 30, seed=5)
        seeds = list(range(100, 112))
        got = {}

        def client(s):
            got[s] = lazy.run_tokens([s % 50], 30, seed=s)
        th = [threading.Thread(target=client, args=(s,)) for s in seeds]
        for t in th:
            t.start()
        for t in th:
            t.join(120)
        assert lazy.wait_captured(120)
        assert all(N.lib().hz_prog_is_captured(q) for q in core.progs + core.progs_lo + core.progs_solo)
        for s in seeds:
            assert got[s] == eager.run_tokens([s % 50], 30, seed=s), s
        assert "deferred_capture_ms" in lazy.timings
    finally:
        eager.close()
        lazy.close()
