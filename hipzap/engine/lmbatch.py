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
from . import lmcore
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
    """pack_lmb's layout written by csrc/pack.hip through the torch-free core (engine/lmcore.py
    ``pack``, shared with the .pth-lite engine hipzap/lmlite.py); same checks, same bytes."""
    emb_src = sd.get("0.encoder.weight")
    dec_w = sd.get("1.decoder.weight")
    tied = dec_w is None or emb_src is None or (
        dec_w.device == emb_src.device and dec_w.data_ptr() == emb_src.data_ptr()
        and dec_w.shape == emb_src.shape and dec_w.stride() == emb_src.stride())
    srcs: dict = {}

    def dev32(k):  # raw fp32 device copy (one H2D; a dtype conversion only for non-fp32 checkpoints)
        if k not in srcs:
            t = sd[k].to(dev, non_blocking=True)
            srcs[k] = (t if t.dtype == torch.float32 else t.float()).contiguous()
        return srcs[k]

    if not tied:
        tied = torch.equal(dev32("1.decoder.weight"), dev32("0.encoder.weight"))
    geo = lmcore.geometry({k: tuple(v.shape) for k, v in sd.items() if hasattr(v, "shape")}, tied=tied)
    layers = []
    for ly in geo.layers:
        w = torch.empty(ly.R // 16, (ly.Kh + ly.Kx) // 32, 64, 8, dtype=torch.bfloat16, device=dev)
        layers.append({"w": w, "bias": torch.empty(ly.R, dtype=torch.float32, device=dev), "H": ly.H, "In": ly.In,
                       "Kh": ly.Kh, "Kx": ly.Kx, "R": ly.R})
    vocab = lambda: torch.empty(geo.Vp // 16, geo.Ke // 32, 64, 8, dtype=torch.bfloat16, device=dev)  # noqa: E731
    embp = vocab()
    decp = embp if geo.dec_key is None else vocab()
    bias = torch.empty(geo.Vp, dtype=torch.float32, device=dev)
    dst = {"layers": [(ly["w"].data_ptr(), ly["bias"].data_ptr()) for ly in layers], "emb": embp.data_ptr(),
           "dec": decp.data_ptr(), "dec_bias": bias.data_ptr()}
    lmcore.pack(geo, lambda k: dev32(k).data_ptr() if k else 0, dst, N.stream_ptr())
    torch.cuda.current_stream(dev).synchronize()  # the fp32 sources are released on return
    return {"layers": layers, "emb": embp, "dec": decp, "dec_bias": bias, "V": geo.V, "Vp": geo.Vp, "E": geo.E,
            "Ke": geo.Ke}


class _TorchAlloc:
    """lmcore allocator over torch tensors (zero-filled device / pinned host bytes)."""

    def __init__(self, dev: torch.device):
        self.dev, self.keep = dev, []

    def device(self, nbytes: int) -> int:
        t = torch.zeros(max(1, nbytes), dtype=torch.uint8, device=self.dev)
        # the fill runs on torch's current stream; LmbCore launches on its own non-blocking stream
        # right after (e.g. lmb_embproj_kernel writing the 1.1 GB projected-embedding table), which
        # is not ordered after it: finish the fill before handing the bytes out
        torch.cuda.current_stream(self.dev).synchronize()
        self.keep.append(t)
        return t.data_ptr()

    def pinned(self, nbytes: int) -> int:
        t = torch.zeros(max(1, nbytes), dtype=torch.uint8, pin_memory=True)
        self.keep.append(t)
        return t.data_ptr()


def geometry_of(packed: dict) -> lmcore.LmbGeometry:
    layers = [lmcore.LmbLayer(ly["H"], ly["In"], ly["Kh"], ly["Kx"], ly["R"], ()) for ly in packed["layers"]]
    return lmcore.LmbGeometry(layers, packed["V"], packed["E"], packed["Ke"], packed["Vp"], None, None)


class LMBatchEngine:
    """``rows`` request rows (16 or 32) decoding together; ``unroll`` steps per captured replay.
    ``generate`` / ``run_tokens`` are thread-safe and block until the request's tokens are out;
    concurrent callers share decode steps. ``record_logits``: keep a pinned [rows, V] buffer so
    ``run_tokens(..., logits=True)`` also returns the logits after the last prompt token."""

    def __init__(self, packed: dict, device="cuda:0", rows: int = 32, unroll: int = 8, exclude_ids=(),
                 max_words: int = 1024, record_logits: bool = False, capture: bool = True,
                 lowload: bool | None = None, embproj: bool | None = None, solo: bool | None = None,
                 priority: int = 0):
        self.p = packed
        self.device = torch.device(device)
        self.V = packed["V"]
        with torch.cuda.device(self.device):
            self.stream = torch.cuda.Stream(self.device, priority=priority)
            self._alloc = _TorchAlloc(self.device)
            w = {"layers": [(ly["w"].data_ptr(), ly["bias"].data_ptr()) for ly in packed["layers"]],
                 "emb": packed["emb"].data_ptr(), "dec": packed["dec"].data_ptr(),
                 "dec_bias": packed["dec_bias"].data_ptr()}
            self.core = lmcore.LmbCore(geometry_of(packed), w, self._alloc, self.stream.cuda_stream, rows=rows,
                                       unroll=unroll, exclude_ids=exclude_ids, max_words=max_words,
                                       record_logits=record_logits, capture=capture, lowload=lowload,
                                       embproj=embproj, solo=solo)
            torch.cuda.synchronize(self.device)
        self.rows, self.unroll, self.max_words = rows, unroll, max_words
        self._ops = self.core._ops

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
        r = self.core.run_tokens(prompt_ids, n_words, seed, logits)
        self.last_latency_ms = self.core.last_latency_ms
        if logits:
            toks, lg = r
            return toks, torch.frombuffer(bytearray(lg), dtype=torch.float32)
        return r

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
        return self.core.stats()

    def close(self) -> None:
        core = getattr(self, "core", None)
        if core is not None:
            core.close()
