"""AWD-LSTM text generation engine on MI355X (GET /inference on the GPU backend).

The reference rebuilds the model and runs 201 CPU forwards per request with autograd on
(main.py:84-103; 8.9 s measured). Here:
  * cold start packs the state_dict once: per layer ``[W_ih | W_hh]`` concatenated,
    gate rows interleaved (unit j -> rows 4j..4j+3), ``b_ih + b_hh`` folded, K padded to a
    multiple of 64 (128-B rows; the kernels predicate the partial last 512-chunk), bf16;
    the tied embedding/decoder matrix is stored once (bf16, padded);
  * split layout (default, profiles/r2_awd_lstm/v3): the recurrent halves W_hh^l h^l_{t-1} + b^l
    of every layer are computed one step AHEAD inside the decoder kernel (bandwidth-bound, so
    they stream at its rate), layer kernels stream W_ih only, and layer 0 is a lookup in
    ``xtab = W_ih^0 . emb^T`` (fp32 [V, 4 H0]) folded into the layer-1 kernel: a step is
    ``L`` kernels (layer 1 with layer 0 and the token, layers 2.., decoder + W_hh rows).
    Classic layout (``HIPZAP_LM_SPLIT=0``): ``L`` fused [W_ih | W_hh] cell kernels + decoder.
  * the argmax sampler is fused into the NEXT step's first kernel (every workgroup reduces the
    decoder's per-workgroup maxima itself). ``unroll`` steps are
    captured into ONE hipGraph (kernel k of step u reads step ``*step + u``; a 1-thread kernel
    advances the counter once per graph). The recurrent state, the step counter, the prompt
    length, the RNG seed and the token sequence all live on the device, so a request is
    ``ceil((P + n - 1) / unroll)`` graph replays, one final sampler launch and a single
    device->host copy. With ``record_draws`` the standalone top-10 tournament sampler runs in
    every step instead (exactness / distribution tests).
  * the SURVEY §5.4 checkpoint rule applies: effective W_hh = ``module.weight_hh_l0`` when
    present, else ``weight_hh_l0_raw``.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import threading

import torch

from .. import _native as N
from ..serve.text import EXCLUDE_TOKENS, NUM_DRAWS, Detokenizer


def _pad_to(n: int, m: int) -> int:
    return int(math.ceil(n / m) * m)


def _interleave(w: torch.Tensor, H: int) -> torch.Tensor:
    """gate-major [4H, K] (i, f, g, o blocks) -> unit-major rows: new row 4j+q = old row q*H + j"""
    return w.reshape(4, H, -1).permute(1, 0, 2).reshape(4 * H, -1)


def _bf16_rows(w: torch.Tensor, ld: int, dev) -> torch.Tensor:
    wp = torch.zeros(w.shape[0], ld, dtype=torch.bfloat16, device=dev)
    wp[:, : w.shape[1]] = w.to(dev, torch.bfloat16)
    return wp


def split_default(layers: list) -> bool:
    """Split mode (csrc/lstm.hip lstm_x_kernel + the decoder's hh_rows): >= 2 layers, <= 4, every
    hidden size <= 1536 (one 3-chunk recurrent row), unless HIPZAP_LM_SPLIT=0."""
    if os.environ.get("HIPZAP_LM_SPLIT", "1") == "0":
        return False
    return 2 <= len(layers) <= 4 and all(ly["H"] <= 1536 for ly in layers)


def pack_awd_lstm(sd: dict, device, split: bool | None = None) -> dict:
    """state_dict (reference key layout) -> device-ready packed tensors.

    classic: per layer ``[W_ih | W_hh]`` in one bf16 matrix (one GEMV per layer kernel).
    split (default when it applies): ``W_ih`` and ``W_hh`` packed apart -- the recurrent GEMVs
    run a step ahead inside the decoder kernel -- and layer 0's input projection becomes the
    fp32 table ``xtab[v] = W_ih^0 . emb[v]`` ([V, 4 H0], exact fp32 from the checkpoint
    weights), so layer 0 needs no weight stream at all."""
    dev = torch.device(device)
    if any(k.endswith("_reverse") for k in sd):
        raise ValueError("bidirectional AWD-LSTM: a bidirectional layer needs the whole sequence, so it cannot "
                         "drive token-by-token generation (GET /inference); use the eager model")
    raw = []
    l = 0
    while f"0.rnns.{l}.module.weight_ih_l0" in sd:
        pre = f"0.rnns.{l}"
        w_ih = sd[f"{pre}.module.weight_ih_l0"].float()
        w_hh = sd.get(f"{pre}.module.weight_hh_l0", sd.get(f"{pre}.weight_hh_l0_raw")).float()
        b = sd[f"{pre}.module.bias_ih_l0"].float() + sd[f"{pre}.module.bias_hh_l0"].float()
        four_h, n_in = w_ih.shape
        raw.append((w_ih, w_hh, b, n_in, four_h // 4))
        l += 1
    if not raw:
        raise ValueError("not an AWD-LSTM state_dict (no 0.rnns.{l}.module.weight_ih_l0)")
    if split is None:
        split = split_default([{"H": H} for *_, H in raw])
    layers = []
    for i, (w_ih, w_hh, b, n_in, H) in enumerate(raw):
        b = b.reshape(4, H).t().reshape(4 * H).to(dev).contiguous()
        if split:
            ldk, ldh = _pad_to(n_in, 64), _pad_to(H, 64)
            layers.append({"w": None if i == 0 else _bf16_rows(_interleave(w_ih, H), ldk, dev),
                           "w_hh": _bf16_rows(_interleave(w_hh, H), ldh, dev), "bias": b, "In": n_in, "H": H,
                           "ldk": ldk, "ldh": ldh})
        else:
            ldk = _pad_to(n_in + H, 64)
            w = _interleave(torch.cat([w_ih, w_hh], dim=1), H)  # [4H, In+H]
            layers.append({"w": _bf16_rows(w, ldk, dev), "bias": b, "In": n_in, "H": H, "ldk": ldk})
    emb = sd["0.encoder.weight"].float()
    V, E = emb.shape
    xtab = None
    if split:
        w_ih0, H0 = raw[0][0], raw[0][4]
        if w_ih0.shape[1] != E:
            raise ValueError("embedding width mismatch")
        with torch.no_grad():
            xtab = (emb.to(dev) @ _interleave(w_ih0, H0).to(dev).t()).contiguous()  # [V, 4 H0] fp32
    # split: the embedding only feeds the (tied) decoder, whose 16-B row loads need K % 8 only --
    # 1000 instead of 1024 columns streams 2.4 % fewer decoder bytes per token
    lde = _pad_to(max(E, layers[-1]["H"]), 8 if split else 64)
    embp = torch.zeros(V, lde, dtype=torch.bfloat16, device=dev)
    embp[:, :E] = emb.to(dev, torch.bfloat16)
    dec_w = sd.get("1.decoder.weight")
    if dec_w is not None and not torch.equal(dec_w.float(), emb):
        decp = torch.zeros(V, lde, dtype=torch.bfloat16, device=dev)
        decp[:, : dec_w.shape[1]] = dec_w.to(dev, torch.bfloat16)
    else:
        decp = embp  # tied (awd_lstm.py:40)
    dec_b = sd.get("1.decoder.bias")
    dec_b = dec_b.float().to(dev) if dec_b is not None else None
    return {"layers": layers, "emb": embp, "dec": decp, "dec_bias": dec_b, "V": V, "E": E, "lde": lde,
            "split": bool(split), "xtab": xtab}


class LMEngine:
    def __init__(self, packed: dict, device="cuda:0", max_steps: int = 1024, exclude_ids=(), record_draws=False,
                 capture: bool = True, unroll: int = 8):
        self.p = packed
        self.device = torch.device(device)
        self.max_steps = max_steps
        lib = N.lib()
        dev = self.device
        with torch.cuda.device(dev):
            self.stream = torch.cuda.Stream(dev)
            L = packed["layers"]
            self.h = [torch.zeros(2, ly["H"], device=dev) for ly in L]
            self.c = [torch.zeros(2, ly["H"], device=dev) for ly in L]
            self.tok_seq = torch.zeros(max_steps + 1, dtype=torch.int32, device=dev)
            self.step = torch.zeros(1, dtype=torch.int32, device=dev)
            self.n_forced = torch.zeros(1, dtype=torch.int32, device=dev)
            self.seed = torch.zeros(1, dtype=torch.int64, device=dev)
            self.logits = torch.zeros(packed["V"], device=dev)
            self.keys = torch.zeros(packed["V"], device=dev)  # logits + Gumbel noise (decoder epilogue)
            self.draws = torch.full((max_steps, NUM_DRAWS), -1, dtype=torch.int32, device=dev) if record_draws else None
            nblk, rpb = C.c_int(), C.c_int()
            lib.hz_decoder_geometry(packed["V"], C.byref(nblk), C.byref(rpb))
            nblk, rpb = nblk.value, rpb.value
            self.bmax_val = torch.empty(nblk, device=dev)  # decoder workgroup maxima -> sampler
            self.bmax_idx = torch.empty(nblk, dtype=torch.int32, device=dev)
            self.bacc_val = torch.empty(nblk, device=dev)  # maxima over acceptable rows (argmax sampler)
            self.bacc_idx = torch.empty(nblk, dtype=torch.int32, device=dev)
            # fused argmax sampler unless draws are recorded (tournament) or forced off
            self.fused_sampler = not record_draws and not os.environ.get("HIPZAP_SAMPLER_TOURNAMENT")
            self.split = bool(packed.get("split"))
            # split mode: pre[l] = W_hh^l . h^l_{t-1} + b^l, written a step ahead by the decoder kernel
            # (measured: hosting layer l's rows in layer l+1's kernel instead, whose input IS h^l_t,
            # made those latency-bound kernels slower by more than the decoder kernel saved --
            # 44.6 vs 42.7 us/token, profiles/r2_awd_lstm/v3)
            self.pre = [torch.empty(4 * ly["H"], device=dev) for ly in L] if self.split else []
            lstm_prms = []
            for i, ly in enumerate(L):
                if self.split and i == 0:
                    continue  # folded into layer 1's kernel (xtab lookup)
                prm = N.LstmParams()
                prm.w, prm.bias = ly["w"].data_ptr(), ly["bias"].data_ptr()
                prm.emb = packed["emb"].data_ptr() if i == 0 else 0
                prm.lde = packed["lde"]
                prm.tok_seq = self.tok_seq.data_ptr()
                prm.x_state = 0 if i == 0 else self.h[i - 1].data_ptr()
                prm.h_state, prm.c_state = self.h[i].data_ptr(), self.c[i].data_ptr()
                prm.step = self.step.data_ptr()
                prm.In, prm.H, prm.ldk = ly["In"], ly["H"], ly["ldk"]
                if i == 0 and prm.In > packed["lde"]:
                    raise ValueError("embedding width mismatch")
                first = i == (1 if self.split else 0)  # the kernel that consumes the token
                if self.split:
                    prm.emb = 0
                    prm.pre = self.pre[i].data_ptr()
                    if i == 1:
                        prm.x_state = 0
                        prm.xtab = packed["xtab"].data_ptr()
                        prm.pre0 = self.pre[0].data_ptr()
                        prm.h0_state, prm.c0_state = self.h[0].data_ptr(), self.c[0].data_ptr()
                        prm.H0 = L[0]["H"]
                if first and self.fused_sampler:
                    prm.n_forced = self.n_forced.data_ptr()
                    prm.bacc_val, prm.bacc_idx = self.bacc_val.data_ptr(), self.bacc_idx.data_ptr()
                    prm.bmax_val, prm.bmax_idx = self.bmax_val.data_ptr(), self.bmax_idx.data_ptr()
                    prm.nblk, prm.V = nblk, packed["V"]
                lstm_prms.append(prm)
            ex = [int(e) for e in exclude_ids][:8]
            d = N.DecoderParams()
            d.w = packed["dec"].data_ptr()
            d.bias = N.ptr(packed["dec_bias"])
            d.h_state, d.step, d.logits = self.h[-1].data_ptr(), self.step.data_ptr(), self.logits.data_ptr()
            d.V, d.H, d.ldk = packed["V"], L[-1]["H"], packed["lde"]
            d.keys, d.seed = self.keys.data_ptr(), self.seed.data_ptr()
            d.bmax_val, d.bmax_idx, d.nblk, d.rpb = self.bmax_val.data_ptr(), self.bmax_idx.data_ptr(), nblk, rpb
            d.bacc_val, d.bacc_idx = self.bacc_val.data_ptr(), self.bacc_idx.data_ptr()
            d.n_exclude = len(ex)
            for i, e in enumerate(ex):
                d.exclude[i] = e
            if self.split:  # the next step's recurrent partials ride in the decoder launch
                d.n_hh = len(L)
                blk = 0
                for i, ly in enumerate(L):
                    d.hh_w[i], d.hh_b[i] = ly["w_hh"].data_ptr(), ly["bias"].data_ptr()
                    d.hh_h[i], d.hh_out[i] = self.h[i].data_ptr(), self.pre[i].data_ptr()
                    d.hh_H[i], d.hh_ld[i] = ly["H"], ly["ldh"]
                    d.hh_blk[i] = blk
                    blk += -(-4 * ly["H"] // N.HH_ROWS)
                d.hh_blk[len(L)] = blk
                d.hh_blocks = blk
            s = N.SamplerParams()
            s.keys, s.tok_seq, s.step = self.keys.data_ptr(), self.tok_seq.data_ptr(), self.step.data_ptr()
            s.bmax_val, s.bmax_idx, s.nblk, s.rpb = d.bmax_val, d.bmax_idx, nblk, rpb
            s.draws = N.ptr(self.draws)
            s.n_forced = self.n_forced.data_ptr()
            s.V = packed["V"]
            s.bacc_val, s.bacc_idx = d.bacc_val, d.bacc_idx  # used when no draw record is requested
            s.n_exclude = len(ex)
            for i, e in enumerate(ex):
                s.exclude[i] = e
            self._final = None
            if self.fused_sampler:  # the last step's token: nothing runs after its decoder
                self._final = N.SamplerParams.from_buffer_copy(s)
                self._final.step_off = -1
            # one step's ops in order (diagnostics: scripts/diag_lm.py)
            self._ops = [("lstm", prm) for prm in lstm_prms] + [("decoder", d)]
            if not self.fused_sampler:
                self._ops.append(("sampler", s))

            def build(reps):
                prog = lib.hz_prog_create()
                for u in range(reps):  # kernels of the u-th step of the graph run step *step + u
                    for kind, prm in self._ops:
                        q = type(prm).from_buffer_copy(prm)
                        q.step_off = u
                        add = {"lstm": lib.hz_prog_add_lstm, "decoder": lib.hz_prog_add_decoder,
                               "sampler": lib.hz_prog_add_sampler}[kind]
                        N.check(add(prog, C.byref(q), 0), "add_" + kind)
                N.check(lib.hz_prog_add_step_bump(prog, self.step.data_ptr(), reps, 0), "add_step_bump")
                if capture:
                    N.check(lib.hz_prog_capture(prog, self.stream.cuda_stream), "capture")
                return prog

            # one step per graph for remainders, `unroll` steps per graph for the bulk of a request:
            # a graph replay costs ~10 us of host/CP time, more than a step's kernel boundaries
            self.prog = build(1)
            self.unroll = max(1, int(unroll)) if capture else 1
            self.prog_multi = build(self.unroll) if self.unroll > 1 else None
            torch.cuda.synchronize(dev)
        self._lock = threading.Lock()

    @classmethod
    def from_state_dict(cls, sd: dict, device="cuda:0", **kw) -> "LMEngine":
        return cls(pack_awd_lstm(sd, device), device, **kw)

    @classmethod
    def for_vocab(cls, sd: dict, stoi: dict, device="cuda:0", **kw) -> "LMEngine":
        ex = [stoi[w] for w in EXCLUDE_TOKENS if w in stoi]
        return cls(pack_awd_lstm(sd, device), device, exclude_ids=ex, **kw)

    def run_tokens(self, prompt_ids: list, n_words: int, seed: int = 0) -> list:
        """Feed ``prompt_ids``, sample ``n_words`` tokens on device; returns sampled ids."""
        P = len(prompt_ids)
        if P < 1:
            raise ValueError("need at least one prompt token")
        total = P + n_words - 1
        if P + n_words > self.max_steps:
            raise ValueError(f"prompt + words ({P + n_words}) exceeds max_steps {self.max_steps}")
        with self._lock, torch.cuda.device(self.device), torch.cuda.stream(self.stream):
            for t in self.h + self.c:
                t.zero_()
            for pre, ly in zip(self.pre, self.p["layers"]):  # W_hh . 0 + b
                pre.copy_(ly["bias"])
            self.step.zero_()
            self.n_forced.fill_(P)
            self.seed.fill_(int(seed) & ((1 << 62) - 1))
            self.tok_seq[:P].copy_(torch.tensor(prompt_ids, dtype=torch.int32), non_blocking=False)
            bulk, rem = divmod(total, self.unroll) if self.prog_multi else (0, total)
            if bulk:
                N.check(N.lib().hz_prog_replay_n(self.prog_multi, self.stream.cuda_stream, bulk), "replay_n")
            if rem:
                N.check(N.lib().hz_prog_replay_n(self.prog, self.stream.cuda_stream, rem), "replay_n")
            if self._final is not None and n_words > 0:
                N.check(N.lib().hz_sampler_launch(C.byref(self._final), self.stream.cuda_stream), "final sampler")
            out = self.tok_seq[P: P + n_words].to("cpu")
        return out.tolist()

    def generate(self, prompt_words, n_words, itos, stoi, seed=None) -> str:
        ids = [stoi.get(w, 0) for w in prompt_words]
        if seed is None:
            seed = int(torch.randint(0, 2**62, (1,)).item())
        toks = self.run_tokens(ids, n_words, seed)
        det = Detokenizer()
        for w in prompt_words:
            det.add_prompt(w)
        for t in toks:
            det.add(itos[t])
        return det.text

    def step_logits(self, prompt_ids: list) -> torch.Tensor:
        """Teacher-forced logits after feeding ``prompt_ids`` (for numerics tests)."""
        self.run_tokens(prompt_ids, 1, 0)
        return self.logits.detach().cpu().clone()

    def __del__(self):
        try:
            for name in ("prog", "prog_multi"):
                if getattr(self, name, None):
                    N.lib().hz_prog_destroy(getattr(self, name))
                    setattr(self, name, None)
        except Exception:
            pass


class LMPool:
    """N independent decode contexts (own stream, recurrent state, token buffer, captured step
    graph) over ONE packed weight set: concurrent GET /inference requests run in parallel instead
    of queueing on one model's lock (SURVEY.md §8 P10 "per-request state buffers make it
    reentrant"). A request takes an idle context, resets its state and returns it when done."""

    def __init__(self, packed: dict, device="cuda:0", contexts: int = 4, **kw):
        import queue
        self.engines = [LMEngine(packed, device, **kw) for _ in range(max(1, contexts))]
        self._idle = queue.Queue()
        for e in self.engines:
            self._idle.put(e)

    @classmethod
    def for_vocab(cls, sd: dict, stoi: dict, device="cuda:0", contexts: int = 4, **kw) -> "LMPool":
        ex = [stoi[w] for w in EXCLUDE_TOKENS if w in stoi]
        return cls(pack_awd_lstm(sd, device), device, contexts, exclude_ids=ex, **kw)

    def _run(self, fn):
        e = self._idle.get()
        try:
            return fn(e)
        finally:
            self._idle.put(e)

    def generate(self, prompt_words, n_words, itos, stoi, seed=None) -> str:
        return self._run(lambda e: e.generate(prompt_words, n_words, itos, stoi, seed))

    def run_tokens(self, prompt_ids: list, n_words: int, seed: int = 0) -> list:
        return self._run(lambda e: e.run_tokens(prompt_ids, n_words, seed))
