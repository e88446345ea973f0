"""Batched AWD-LSTM text generation: continuous batching of concurrent GET /inference requests.

The reference serves each request in its own Lambda container, rebuilding the model and running
201 CPU forwards per request (/root/reference/main.py:84-112). The single-request
GPU engine (engine/lm.py) replays a captured decode step per token, but every token of every
request streams all ~150 MB of weights. Here ``rows`` requests (16 or 32) share each decode step:
the layers and the decoder run as skinny GEMMs on the matrix cores over all rows at once
(csrc/lmbatch.hip), so the weights are read once per step for every request in flight, and a
native scheduler (csrc/lmserve.cpp) admits new requests into free rows at every replay boundary
(``unroll`` steps per captured graph) and returns each request's tokens as soon as its last one
is sampled.

Semantics per request are the reference's (main.py:40-81): the prompt is fed token by token,
then each step keeps the first of 10 draws without replacement ∝ exp(logits) that is acceptable
(id != 0, not xxup/xxfld/xxrep) -- computed exactly as the argmax of Gumbel-perturbed logits over
the acceptable ids (csrc/lstm.hip sample_argmax), with the same Philox noise (seed, step, id) as
the single-request engine. The checkpoint rules are engine/lm.py's (effective
W_hh = ``module.weight_hh_l0``, tied embedding/decoder).
"""
from __future__ import annotations

import ctypes as C
import math

import torch

from .. import _native as N
from ..serve.text import EXCLUDE_TOKENS, Detokenizer
from .lm import _interleave


def _pad(n: int, m: int) -> int:
    return int(math.ceil(n / m) * m)


def frag_pack(w: torch.Tensor) -> torch.Tensor:
    """[R, K] (R % 16 == 0, K % 32 == 0) -> fragment-major bf16 [R/16][K/32][64][8]: lane l of
    fragment (tile, ks) holds row 16 tile + (l & 15), k = 32 ks + 8 (l >> 4) + j -- the A operand
    of mfma_f32_16x16x32_bf16, one contiguous 1 KiB per wave load."""
    R, K = w.shape
    assert R % 16 == 0 and K % 32 == 0, (R, K)
    t = w.to(torch.bfloat16).reshape(R // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4)
    return t.reshape(R // 16, K // 32, 64, 8).contiguous()


def state_unpack(buf: torch.Tensor, K: int, Bp: int) -> torch.Tensor:
    """One [K/32][Bp/16][64][8] state image -> [Bp, K] (tests / diagnostics)."""
    t = buf.reshape(K // 32, Bp // 16, 4, 16, 8).permute(1, 3, 0, 2, 4)
    return t.reshape(Bp, K)


def _native_pack_ok(dev: torch.device) -> bool:
    if dev.type != "cuda":
        return False
    try:
        return hasattr(N.lib(), "hz_frag_pack_launch")
    except OSError:
        return False


def pack_lmb(sd: dict, device, native: bool | None = None) -> dict:
    """state_dict (reference key layout, awd_lstm.py:7-14) -> the batched engine's weights.

    Per layer l: ``W = [W_hh | W_ih]`` with rows unit-interleaved (row 4j + q = gate q of unit j,
    so one MFMA accumulator holds a unit's four gates), K segments padded to 32 (the last layer's
    recurrent segment to 256: it is also the decoder's K), fragment-major bf16; bias b_ih + b_hh.
    Embedding and decoder: [V, E] padded to [16, 256] multiples, fragment-major, stored once when
    tied (awd_lstm.py:40).

    ``native`` (default on a GPU): the gathers, zero padding, RNE bf16 rounding and bias adds run
    in one own kernel per matrix (csrc/pack.hip ``hz_frag_pack_launch``) on the raw fp32 tensors,
    bitwise the torch ops' result. Measured cold in a fresh process (``scripts/diag_lm_build.py``):
    the torch-op packing is ~280 ms of first-use kernel loading for ~1 ms of work."""
    dev = torch.device(device)
    if native is None:
        native = _native_pack_ok(dev)
    if native:
        return _pack_lmb_native(sd, dev)
    if any(k.endswith("_reverse") for k in sd):
        raise ValueError("bidirectional AWD-LSTM cannot drive token-by-token generation")
    emb = sd["0.encoder.weight"].float()
    V, E = emb.shape
    Ke = _pad(E, 256)
    if Ke > 1024:
        raise ValueError(f"batched decode supports embedding widths <= 1024 (got {E})")
    raw = []
    l = 0
    while f"0.rnns.{l}.module.weight_ih_l0" in sd:
        pre = f"0.rnns.{l}"
        w_ih = sd[f"{pre}.module.weight_ih_l0"].float()
        w_hh = sd.get(f"{pre}.module.weight_hh_l0", sd.get(f"{pre}.weight_hh_l0_raw")).float()
        b = sd[f"{pre}.module.bias_ih_l0"].float() + sd[f"{pre}.module.bias_hh_l0"].float()
        raw.append((w_ih, w_hh, b, w_ih.shape[1], w_ih.shape[0] // 4))
        l += 1
    if not raw:
        raise ValueError("not an AWD-LSTM state_dict (no 0.rnns.{l}.module.weight_ih_l0)")
    if len(raw) > 4:
        raise ValueError("batched decode supports up to 4 layers")
    if raw[0][3] != E or raw[-1][4] != E:
        raise ValueError("batched decode needs layer 0 input and last hidden size = embedding width (tied model)")
    layers = []
    for i, (w_ih, w_hh, b, n_in, H) in enumerate(raw):
        Kh = Ke if i == len(raw) - 1 else _pad(H, 32)
        Kx = Ke if i == 0 else layers[-1]["Kh"]
        R = _pad(4 * H, 16)
        w = torch.zeros(R, Kh + Kx, device=dev)
        w[: 4 * H, :H] = _interleave(w_hh.to(dev), H)
        w[: 4 * H, Kh: Kh + n_in] = _interleave(w_ih.to(dev), H)
        bias = torch.zeros(R, device=dev)
        bias[: 4 * H] = b.reshape(4, H).t().reshape(4 * H).to(dev)
        if (Kh + Kx) // 32 > 72:
            raise ValueError(f"layer {i}: K = {Kh + Kx} exceeds the batched kernel's 2304")
        layers.append({"w": frag_pack(w), "bias": bias.contiguous(), "H": H, "In": n_in, "Kh": Kh, "Kx": Kx, "R": R})
    Vp = _pad(V, 16)

    def pack_vocab(m: torch.Tensor) -> torch.Tensor:
        t = torch.zeros(Vp, Ke, device=dev)
        t[:V, : m.shape[1]] = m.to(dev)
        return frag_pack(t)

    embp = pack_vocab(emb)
    dec_w = sd.get("1.decoder.weight")
    decp = embp if dec_w is None or torch.equal(dec_w.float(), emb) else pack_vocab(dec_w.float())
    dec_b = sd.get("1.decoder.bias")
    bias = torch.zeros(Vp, device=dev)
    if dec_b is not None:
        bias[:V] = dec_b.float().to(dev)
    return {"layers": layers, "emb": embp, "dec": decp, "dec_bias": bias, "V": V, "Vp": Vp, "E": E, "Ke": Ke}


def _lmb_layers(sd: dict) -> list:
    """(w_ih, w_hh, b_ih, b_hh, n_in, H) per layer, as stored (the effective W_hh rule of pack_lmb)."""
    raw = []
    l = 0
    while f"0.rnns.{l}.module.weight_ih_l0" in sd:
        pre = f"0.rnns.{l}"
        w_ih = sd[f"{pre}.module.weight_ih_l0"]
        w_hh = sd.get(f"{pre}.module.weight_hh_l0", sd.get(f"{pre}.weight_hh_l0_raw"))
        raw.append((w_ih, w_hh, sd[f"{pre}.module.bias_ih_l0"], sd[f"{pre}.module.bias_hh_l0"], w_ih.shape[1],
                    w_ih.shape[0] // 4))
        l += 1
    return raw


def _pack_lmb_native(sd: dict, dev: torch.device) -> dict:
    """pack_lmb's layout written by csrc/pack.hip (see pack_lmb); same checks, same bytes."""
    if any(k.endswith("_reverse") for k in sd):
        raise ValueError("bidirectional AWD-LSTM cannot drive token-by-token generation")
    emb_src = sd["0.encoder.weight"]
    V, E = emb_src.shape
    Ke = _pad(E, 256)
    if Ke > 1024:
        raise ValueError(f"batched decode supports embedding widths <= 1024 (got {E})")
    raw = _lmb_layers(sd)
    if not raw:
        raise ValueError("not an AWD-LSTM state_dict (no 0.rnns.{l}.module.weight_ih_l0)")
    if len(raw) > 4:
        raise ValueError("batched decode supports up to 4 layers")
    if raw[0][4] != E or raw[-1][5] != E:
        raise ValueError("batched decode needs layer 0 input and last hidden size = embedding width (tied model)")

    def dev32(t):  # raw fp32 device copy (one H2D; a dtype conversion only for non-fp32 checkpoints)
        t = t.to(dev, non_blocking=True)
        return (t if t.dtype == torch.float32 else t.float()).contiguous()

    lib = N.lib()
    st = N.stream_ptr()

    def launch(**kw):
        p = N.FragPackParams()
        for k, v in kw.items():
            setattr(p, k, v.data_ptr() if isinstance(v, torch.Tensor) else v)
        N.check(lib.hz_frag_pack_launch(C.byref(p), st), "hz_frag_pack_launch")

    layers = []
    for i, (w_ih, w_hh, b_ih, b_hh, n_in, H) in enumerate(raw):
        Kh = Ke if i == len(raw) - 1 else _pad(H, 32)
        Kx = Ke if i == 0 else layers[-1]["Kh"]
        R = _pad(4 * H, 16)
        if (Kh + Kx) // 32 > 72:
            raise ValueError(f"layer {i}: K = {Kh + Kx} exceeds the batched kernel's 2304")
        a, b, ba, bb = dev32(w_hh), dev32(w_ih), dev32(b_ih), dev32(b_hh)
        w = torch.empty(R // 16, (Kh + Kx) // 32, 64, 8, dtype=torch.bfloat16, device=dev)
        bias = torch.empty(R, dtype=torch.float32, device=dev)
        launch(a=a, b=b, out=w, bias_a=ba, bias_b=bb, bias_out=bias, R=R, K=Kh + Kx, nrows=4 * H, interleave_h=H,
               ka=Kh, acols=H, lda=H, bcols=n_in, ldb=n_in)
        layers.append({"w": w, "bias": bias, "H": H, "In": n_in, "Kh": Kh, "Kx": Kx, "R": R, "_src": (a, b, ba, bb)})
    Vp = _pad(V, 16)
    emb = dev32(emb_src)

    def pack_vocab(m):
        t = torch.empty(Vp // 16, Ke // 32, 64, 8, dtype=torch.bfloat16, device=dev)
        launch(a=m, out=t, R=Vp, K=Ke, nrows=V, ka=Ke, acols=E, lda=E)
        return t

    embp = pack_vocab(emb)
    dec_w = sd.get("1.decoder.weight")
    tied = dec_w is None or (dec_w.device == emb_src.device and dec_w.data_ptr() == emb_src.data_ptr()
                             and dec_w.shape == emb_src.shape and dec_w.stride() == emb_src.stride())
    dec = None
    if not tied:
        dec = dev32(dec_w)
        tied = torch.equal(dec, emb)
    decp = embp if tied else pack_vocab(dec)
    dec_b = sd.get("1.decoder.bias")
    dbias = dev32(dec_b) if dec_b is not None else None
    bias = torch.empty(Vp, dtype=torch.float32, device=dev)
    launch(bias_a=dbias if dbias is not None else 0, bias_out=bias, R=Vp, K=32, nrows=V, ka=32)
    torch.cuda.current_stream(dev).synchronize()  # the fp32 sources are released on return
    for ly in layers:
        del ly["_src"]
    return {"layers": layers, "emb": embp, "dec": decp, "dec_bias": bias, "V": V, "Vp": Vp, "E": E, "Ke": Ke}


class LMBatchEngine:
    """``rows`` request rows (16 or 32) decoding together; ``unroll`` steps per captured replay.
    ``generate`` / ``run_tokens`` are thread-safe and block until the request's tokens are out;
    concurrent callers share decode steps. ``record_logits``: keep a pinned [rows, V] buffer so
    ``run_tokens(..., logits=True)`` also returns the logits after the last prompt token."""

    def __init__(self, packed: dict, device="cuda:0", rows: int = 32, unroll: int = 8, exclude_ids=(),
                 max_words: int = 1024, record_logits: bool = False, capture: bool = True):
        if rows not in (16, 32):
            raise ValueError("rows must be 16 or 32")
        if not 1 <= unroll <= 32:
            raise ValueError("unroll must be in 1..32")
        self.p = packed
        self.device = torch.device(device)
        self.rows, self.unroll, self.max_words = rows, unroll, max_words
        self.V = packed["V"]
        lib = N.lib()
        dev, Bp, U = self.device, rows, unroll
        L = packed["layers"]
        with torch.cuda.device(dev):
            self.stream = torch.cuda.Stream(dev)
            self.h = [torch.zeros(4 * ly["Kh"] * Bp, dtype=torch.int16, device=dev) for ly in L]
            self.c = [torch.zeros(Bp * ly["H"], device=dev) for ly in L]
            self.gpar = torch.zeros(1, dtype=torch.int32, device=dev)
            self.ctl = torch.zeros(U * Bp * 4, dtype=torch.int32, device=dev)
            self.seed = torch.zeros(Bp, dtype=torch.int64, device=dev)
            self.outp = torch.zeros(Bp, dtype=torch.int64, device=dev)
            self.nblk = lib.hz_lmb_dec_blocks(self.V)
            self.dbest = torch.zeros(2 * Bp, dtype=torch.int64, device=dev)  # [parity][row]
            self.tok = torch.zeros(Bp, dtype=torch.int32, device=dev)
            self.block = torch.zeros(8 + Bp * (8 + 4 * U), dtype=torch.int32, pin_memory=True)
            self.out_pool = torch.zeros(Bp * max_words, dtype=torch.int32, pin_memory=True)
            self.logits = torch.zeros(Bp * self.V, dtype=torch.float32, pin_memory=True) if record_logits else None
            ex = [int(e) for e in exclude_ids][:8]

            a = N.LmbAdmitParams()
            a.block, a.ctl, a.seed, a.outp, a.gpar = (self.block.data_ptr(), self.ctl.data_ptr(),
                                                      self.seed.data_ptr(), self.outp.data_ptr(), self.gpar.data_ptr())
            a.Bp, a.U, a.n_layers = Bp, U, len(L)
            for i, ly in enumerate(L):
                a.h[i], a.c[i], a.Kh[i], a.H[i] = self.h[i].data_ptr(), self.c[i].data_ptr(), ly["Kh"], ly["H"]
            layer_prms = []
            for i, ly in enumerate(L):
                q = N.LmbLayerParams()
                q.w, q.bias, q.h, q.c = ly["w"].data_ptr(), ly["bias"].data_ptr(), self.h[i].data_ptr(), self.c[i].data_ptr()
                q.x = 0 if i == 0 else self.h[i - 1].data_ptr()
                q.gpar, q.ctl = self.gpar.data_ptr(), self.ctl.data_ptr()
                q.H, q.Kh, q.Kx, q.R, q.Bp = ly["H"], ly["Kh"], ly["Kx"], ly["R"], Bp
                if i == 0:
                    q.emb, q.dbest, q.V = packed["emb"].data_ptr(), self.dbest.data_ptr(), self.V
                    q.outp, q.tok = self.outp.data_ptr(), self.tok.data_ptr()
                layer_prms.append(q)
            d = N.LmbDecParams()
            d.w, d.bias, d.h = packed["dec"].data_ptr(), packed["dec_bias"].data_ptr(), self.h[-1].data_ptr()
            d.gpar, d.ctl, d.seed, d.dbest = self.gpar.data_ptr(), self.ctl.data_ptr(), self.seed.data_ptr(), self.dbest.data_ptr()
            d.logits = self.logits.data_ptr() if self.logits is not None else 0
            d.V, d.Vp, d.K, d.Bp, d.nblk = self.V, packed["Vp"], L[-1]["Kh"], Bp, self.nblk
            d.n_exclude = len(ex)
            for i, e in enumerate(ex):
                d.exclude[i] = e
            self._ops = [(N.HZ_K_LMB_LAYER, q) for q in layer_prms] + [(N.HZ_K_LMB_DEC, d)]
            prog = lib.hz_prog_create()
            N.check(lib.hz_prog_add_kernel(prog, N.HZ_K_LMB_ADMIT, C.byref(a), C.sizeof(a), 0), "add lmb admit")
            for u in range(U):
                for kind, prm in self._ops:
                    q = type(prm).from_buffer_copy(prm)
                    q.step_off = u
                    N.check(lib.hz_prog_add_kernel(prog, kind, C.byref(q), C.sizeof(q), 0), f"add lmb kernel {kind}")
            self._admit = a
            self.prog = prog
            if capture:
                N.check(lib.hz_prog_capture(prog, self.stream.cuda_stream), "capture lmb")
            torch.cuda.synchronize(dev)
        self._sched = lib.hz_lmb_create(prog, self.stream.cuda_stream, self.block.data_ptr(), Bp, U, 0, max_words,
                                        self.out_pool.data_ptr(), d.logits, self.V)
        if not self._sched:
            raise RuntimeError("hz_lmb_create failed")

    @classmethod
    def from_state_dict(cls, sd: dict, device="cuda:0", **kw) -> "LMBatchEngine":
        return cls(pack_lmb(sd, device), device, **kw)

    @classmethod
    def for_vocab(cls, sd: dict, stoi: dict, device="cuda:0", **kw) -> "LMBatchEngine":
        ex = [stoi[w] for w in EXCLUDE_TOKENS if w in stoi]
        return cls(pack_lmb(sd, device), device, exclude_ids=ex, **kw)

    def run_tokens(self, prompt_ids: list, n_words: int, seed: int = 0, logits: bool = False):
        """Feed ``prompt_ids``, sample ``n_words`` tokens; returns the sampled ids (and, with
        ``logits``, the fp32 logits after the last prompt token)."""
        P = len(prompt_ids)
        if P < 1:
            raise ValueError("need at least one prompt token")
        if not 1 <= n_words <= self.max_words:
            raise ValueError(f"n_words must be in 1..{self.max_words}")
        if logits and self.logits is None:
            raise ValueError("engine built without record_logits")
        prompt = (C.c_int * P)(*[int(t) for t in prompt_ids])
        out = (C.c_int * n_words)()
        lg = (C.c_float * self.V)() if logits else None
        lat = C.c_double()
        rc = N.lib().hz_lmb_submit(self._sched, prompt, P, n_words, int(seed) & ((1 << 62) - 1), out,
                                   lg, C.byref(lat))
        if rc:
            raise RuntimeError(f"batched decode request failed ({rc})")
        self.last_latency_ms = lat.value / 1e3
        toks = list(out)
        if logits:
            return toks, torch.frombuffer(bytearray(lg), dtype=torch.float32)
        return toks

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

    def stats(self) -> dict:
        a = (C.c_uint64 * 4)()
        N.lib().hz_lmb_stats(self._sched, a)
        return {"replays": a[0], "served": a[1], "row_steps_used": a[2], "row_steps": a[3],
                "row_utilisation": round(a[2] / a[3], 4) if a[3] else None}

    def close(self) -> None:
        s, self._sched = getattr(self, "_sched", None), None
        if s:
            N.lib().hz_lmb_destroy(s)
        prog, self.prog = getattr(self, "prog", None), None
        if prog:
            N.lib().hz_prog_destroy(prog)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
