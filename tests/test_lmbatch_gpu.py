"""Batched AWD-LSTM decode (engine/lmbatch.py, csrc/lmbatch.hip + csrc/lmserve.cpp) on the GPU:
logits vs the eager fp32 model and the single-request engine, exactness of the sampled token
(argmax of Gumbel keys over acceptable ids, host-recomputed Philox noise), and row independence:
a request's tokens are bitwise the same whether it runs alone or shares steps with 40 others."""
import threading

import numpy as np
import pytest
import torch

from hipzap.engine.lm import LMEngine, pack_awd_lstm
from hipzap.engine.lmbatch import LMBatchEngine, pack_lmb
from hipzap.models.awd_lstm import get_language_model, reference_lm

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def model():
    torch.manual_seed(0)
    return reference_lm(3000).eval()  # the reference's dims (emb 1000, hidden 1150, 3 layers), small vocab


@pytest.fixture(scope="module")
def engine(model):
    eng = LMBatchEngine(pack_lmb(model.state_dict(), DEV), DEV, rows=32, unroll=8, exclude_ids=[2, 5],
                        record_logits=True)
    yield eng
    eng.close()


def _eager_logits(m, ids):
    m.reset()
    with torch.no_grad():
        for t in ids:
            res, *_ = m(torch.tensor([[t]]))
    return res[-1]


def gumbel_np(seed: int, t: int, V: int) -> np.ndarray:
    """Host copy of common.h gumbel(seed, t, j) for j = 0..V-1 (Philox4x32-10, one block per 4 ids)."""
    M = np.uint64(0xFFFFFFFF)
    j = np.arange(V, dtype=np.uint64)
    c0 = j >> np.uint64(2)
    c1 = np.full(V, t & 0xFFFFFFFF, np.uint64)
    c2 = np.full(V, 0x5EED, np.uint64)
    c3 = np.zeros(V, np.uint64)
    k0, k1 = np.uint64(seed & 0xFFFFFFFF), np.uint64((seed >> 32) & 0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c0
        p1 = np.uint64(0xCD9E8D57) * c2
        h0, l0 = p0 >> np.uint64(32), p0 & M
        h1, l1 = p1 >> np.uint64(32), p1 & M
        c0, c1, c2, c3 = h1 ^ c1 ^ k0, l1, h0 ^ c3 ^ k1, l0
        k0 = (k0 + np.uint64(0x9E3779B9)) & M
        k1 = (k1 + np.uint64(0xBB67AE85)) & M
    r = np.choose((j & np.uint64(3)).astype(np.int64), [c0, c1, c2, c3])
    u = ((r >> np.uint64(8)).astype(np.float64) + 0.5) / 16777216.0
    return -np.log(-np.log(u))


@pytest.mark.parametrize("unroll", [1, 8])
def test_teacher_forced_logits_match_eager_and_single_engine(model, unroll):
    eng = LMBatchEngine(pack_lmb(model.state_dict(), DEV), DEV, rows=16, unroll=unroll, record_logits=True)
    single = LMEngine(pack_awd_lstm(model.state_dict(), DEV), DEV)
    try:
        for ids in ([5], [5, 17, 200, 3, 2999], [9, 8, 7, 6, 5, 4, 3, 2, 1, 11, 12]):
            _, got = eng.run_tokens(ids, 1, seed=1, logits=True)
            ref = _eager_logits(model, ids)
            rel = (got - ref).abs().max().item() / ref.abs().max().item()
            assert rel < 3e-2, rel
            assert int(got.argmax()) == int(ref.argmax())
            # vs the single-request engine (fp32 state, same bf16 weights): the hi/lo state pair keeps
            # the batched recurrence within a few e-3 of it
            one = single.step_logits(ids)
            assert (got - one).abs().max().item() / one.abs().max().item() < 1e-2
    finally:
        eng.close()


def test_sampled_token_is_argmax_of_acceptable_keys(engine):
    """The token of each step = argmax over acceptable ids of logit + Gumbel(seed, t, id) (the
    main.py:63-68 rule, exactly), recomputed on the host from the recorded logits."""
    ids = [11, 12, 13]
    for seed in range(6):
        toks, lg = engine.run_tokens(ids, 1, seed=seed, logits=True)
        keys = lg.double().numpy() + gumbel_np(seed, len(ids) - 1, lg.numel())
        keys[[0, 2, 5]] = -np.inf  # id 0 + the engine's excluded ids
        best = int(np.argmax(keys))
        assert toks[0] == best or keys[toks[0]] >= keys[best] - 1e-4, (toks[0], best)


def test_requests_are_independent_of_the_batch(engine):
    """40 concurrent requests (mixed prompt lengths, seeds, lengths; more than the 32 rows, so
    some wait and join mid-stream) give bitwise the tokens each gives alone."""
    rng = np.random.default_rng(0)
    jobs = [([int(x) for x in rng.integers(1, 3000, int(rng.integers(1, 6)))], int(rng.integers(5, 60)), s)
            for s in range(40)]
    alone = [engine.run_tokens(p, n, seed=s) for p, n, s in jobs]
    out = [None] * len(jobs)

    def go(i):
        p, n, s = jobs[i]
        out[i] = engine.run_tokens(p, n, seed=s)

    th = [threading.Thread(target=go, args=(i,)) for i in range(len(jobs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert out == alone
    assert all(len(o) == n for o, (_, n, _) in zip(out, jobs))
    st = engine.stats()
    assert st["served"] >= 80 and st["row_utilisation"] > 0


def test_lowload_program_is_bitwise_the_full_one(model):
    """A lone request (every busy row below 16) replays the 16-row program (csrc/lmserve.cpp
    low load); its tokens and logits are bitwise those of the full 32-row program."""
    pk = pack_lmb(model.state_dict(), DEV)
    full = LMBatchEngine(pk, DEV, rows=32, unroll=8, exclude_ids=[2], record_logits=True, lowload=False,
                         solo=False)
    low = LMBatchEngine(pk, DEV, rows=32, unroll=8, exclude_ids=[2], record_logits=True, lowload=True,
                        solo=False)
    try:
        for seed, (ids, n) in enumerate([([4, 7], 30), ([9] * 9, 17), ([123], 1)]):
            a, la = full.run_tokens(ids, n, seed=seed, logits=True)
            b, lb = low.run_tokens(ids, n, seed=seed, logits=True)
            assert a == b and torch.equal(la, lb)
        assert low.stats()["lowload_replays"] > 0 and full.stats()["lowload_replays"] == 0
    finally:
        full.close()
        low.close()


@pytest.mark.parametrize("rows", [16, 32])
def test_one_request_program_is_bitwise_the_full_one(model, rows):
    """A lone request (row 0 the only busy row) replays the one-request program (nb_act = -1:
    the kernels read and write row 0's state only); its tokens and logits are bitwise those of
    the full program, and requests that join while it runs switch programs without a change."""
    pk = pack_lmb(model.state_dict(), DEV)
    full = LMBatchEngine(pk, DEV, rows=rows, unroll=8, exclude_ids=[2], record_logits=True, lowload=False,
                         solo=False)
    one = LMBatchEngine(pk, DEV, rows=rows, unroll=8, exclude_ids=[2], record_logits=True, solo=True)
    try:
        for seed, (ids, n) in enumerate([([4, 7], 30), ([9] * 9, 17), ([123], 1)]):
            a, la = full.run_tokens(ids, n, seed=seed, logits=True)
            b, lb = one.run_tokens(ids, n, seed=seed, logits=True)
            assert a == b and torch.equal(la, lb)
        assert one.stats()["solo_replays"] > 0 and full.stats()["solo_replays"] == 0
        # a long request alone, then others joining (and leaving) while it runs
        jobs = [([5, 6], 120, 100)] + [([int(3 + i)], 20 + 3 * i, 200 + i) for i in range(6)]
        ref = [full.run_tokens(p, n, seed=s) for p, n, s in jobs]
        out = [None] * len(jobs)

        def go(i):
            p, n, s = jobs[i]
            out[i] = one.run_tokens(p, n, seed=s)

        th = [threading.Thread(target=go, args=(0,))]
        th[0].start()
        import time
        time.sleep(0.002)
        th += [threading.Thread(target=go, args=(i,)) for i in range(1, len(jobs))]
        for t in th[1:]:
            t.start()
        for t in th:
            t.join()
        assert out == ref
    finally:
        full.close()
        one.close()


def test_projected_embedding_matches_the_fused_first_layer(model):
    """HIPZAP_LM_EMBPROJ: the first layer's embedding half precomputed per vocabulary id (fp32
    W_ih E[v], lmb_embproj_kernel) gives the logits of the engine that multiplies it every step,
    up to fp32 summation order."""
    pk = pack_lmb(model.state_dict(), DEV)
    a = LMBatchEngine(pk, DEV, rows=32, unroll=8, record_logits=True, embproj=False)
    b = LMBatchEngine(pk, DEV, rows=32, unroll=8, record_logits=True, embproj=True)
    try:
        assert b.core.embproj and not a.core.embproj
        for ids in ([5], [5, 17, 200, 3, 2999], [9, 8, 7, 6, 5, 4, 3, 2, 1, 11, 12]):
            _, la = a.run_tokens(ids, 1, seed=1, logits=True)
            _, lb = b.run_tokens(ids, 1, seed=1, logits=True)
            assert (la - lb).abs().max().item() / la.abs().max().item() < 2e-3
        agree = sum(a.run_tokens([4, 7], 10, seed=s) == b.run_tokens([4, 7], 10, seed=s) for s in range(10))
        assert agree >= 9, agree
    finally:
        a.close()
        b.close()


def test_tokens_track_the_single_request_engine(model):
    """Same seed, same rule, same noise: the batched engine's tokens agree with the single-request
    engine's (fp32 state) except where two keys are closer than the small state rounding."""
    excl = [2]
    eng = LMBatchEngine(pack_lmb(model.state_dict(), DEV), DEV, rows=32, unroll=8, exclude_ids=excl)
    single = LMEngine(pack_awd_lstm(model.state_dict(), DEV), DEV, exclude_ids=excl)
    try:
        agree = 0
        for seed in range(20):
            a = eng.run_tokens([4, 7], 10, seed=seed)
            b = single.run_tokens([4, 7], 10, seed=seed)
            agree += a == b
        assert agree >= 17, agree
    finally:
        eng.close()


def test_reference_dims_v60000_generate():
    """The reference's serving configuration (emb 1000, hidden 1150, 3 layers, tied, V=60000):
    logits vs eager fp32, then 200-word requests from the empty prompt (main.py:103)."""
    torch.manual_seed(3)
    m = reference_lm(60000).eval()
    itos = [f"w{i}" for i in range(60000)]
    itos[0], itos[1], itos[2] = "xxunk", "xxpad", "."
    stoi = {w: i for i, w in enumerate(itos)}
    eng = LMBatchEngine.for_vocab(m.state_dict(), stoi, DEV, rows=32, unroll=8, record_logits=True)
    try:
        ids = [7, 59999, 123, 40000]
        _, got = eng.run_tokens(ids, 1, seed=0, logits=True)
        ref = _eager_logits(m, ids)
        assert (got - ref).abs().max().item() / ref.abs().max().item() < 3e-2
        assert int(got.argmax()) == int(ref.argmax())
        a = eng.generate([""], 200, itos, stoi, seed=7)
        b = eng.generate([""], 200, itos, stoi, seed=7)
        assert a == b and len(a.split()) >= 150
    finally:
        eng.close()


def test_untied_two_layer_model():
    torch.manual_seed(1)
    m = get_language_model(vocab_sz=700, emb_sz=96, n_hid=160, n_layers=2, pad_token=1, tie_weights=False).eval()
    eng = LMBatchEngine.from_state_dict(m.state_dict(), DEV, rows=16, unroll=4, record_logits=True)
    try:
        ids = [3, 9, 650]
        _, got = eng.run_tokens(ids, 1, logits=True)
        ref = _eager_logits(m, ids)
        assert (got - ref).abs().max().item() / ref.abs().max().item() < 3e-2
    finally:
        eng.close()


def _packs_equal(a: dict, b: dict) -> None:
    assert [k for k in a] == [k for k in b]
    for k in ("V", "Vp", "E", "Ke"):
        assert a[k] == b[k], k
    for k in ("emb", "dec", "dec_bias"):
        assert a[k].dtype == b[k].dtype and torch.equal(a[k].view(torch.int16) if a[k].dtype == torch.bfloat16 else a[k],
                                                        b[k].view(torch.int16) if b[k].dtype == torch.bfloat16 else b[k]), k
    assert (a["dec"] is a["emb"]) == (b["dec"] is b["emb"])  # tied stays stored once
    for la, lb in zip(a["layers"], b["layers"]):
        assert {k: v for k, v in la.items() if not torch.is_tensor(v)} == {k: v for k, v in lb.items() if not torch.is_tensor(v)}
        assert torch.equal(la["w"].view(torch.int16), lb["w"].view(torch.int16)) and torch.equal(la["bias"], lb["bias"])


@pytest.mark.parametrize("case", ["reference_tied", "untied_biased_two_layer", "bf16_checkpoint", "on_device_sd"])
def test_native_pack_is_bitwise_the_torch_pack(model, case):
    """csrc/pack.hip hz_frag_pack_launch (the GPU default) writes exactly pack_lmb's torch-op
    bytes: unit-interleaved gate rows, [W_hh | W_ih] segments with zero padding, RNE bf16, b_ih +
    b_hh in fp32, the vocabulary matrix padded to [16, 256] multiples, tied weights stored once."""
    if case == "reference_tied":
        sd = model.state_dict()
    elif case == "untied_biased_two_layer":
        torch.manual_seed(2)
        m = get_language_model(vocab_sz=700, emb_sz=96, n_hid=160, n_layers=2, pad_token=1, tie_weights=False).eval()
        sd = m.state_dict()
        if "1.decoder.bias" in sd:
            sd["1.decoder.bias"] = torch.randn_like(sd["1.decoder.bias"])
    elif case == "bf16_checkpoint":
        sd = {k: (v.to(torch.bfloat16) if v.is_floating_point() else v) for k, v in model.state_dict().items()}
    else:
        sd = {k: v.to(DEV) for k, v in model.state_dict().items()}
    _packs_equal(pack_lmb(sd, DEV, native=False), pack_lmb(sd, DEV, native=True))
