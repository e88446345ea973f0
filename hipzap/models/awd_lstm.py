"""AWD-LSTM language model — the reference's model (checkpoint-compatible).

Behavioural contract taken from the reference (read, not copied):
  * factory ``get_language_model(vocab_sz, emb_sz, n_hid, n_layers, pad_token, tie_weights,
    qrnn, bias, bidir, output_p, hidden_p, input_p, embed_p, weight_p)``
    (/root/reference/pytorch_models/awd_lstm.py:7-14), returning a 2-element sequential
    model: ``[0]`` the recurrent core, ``[1]`` the linear decoder, with ``reset()``;
  * sequence-first input ``LongTensor[sl, bs]``; ``forward`` returns
    ``(decoded[sl*bs, V], raw_outputs, outputs)`` (awd_lstm.py:42-46, 77-91);
  * hidden state persists across calls, is detached each call and is re-initialised when the
    batch size changes (awd_lstm.py:79-81, 90);
  * layer l maps emb->n_hid ... n_hid->emb so the decoder can share the embedding matrix
    (awd_lstm.py:69-72, 40);
  * eval-mode dropouts are identities; training-mode semantics: locked (variational)
    dropout over the sequence axis, whole-row embedding dropout, DropConnect on W_hh.
  * state_dict keys: ``0.encoder.weight``, ``0.encoder_dp.emb.weight``,
    ``0.rnns.{l}.weight_hh_l0_raw``, ``0.rnns.{l}.module.{weight_ih_l0,weight_hh_l0,
    bias_ih_l0,bias_hh_l0}``, ``1.decoder.{weight,bias}``; the effective W_hh after loading
    is the checkpoint's ``module.weight_hh_l0`` (falls back to ``_raw``), the SURVEY §5.4 quirk.
The QRNN branch of the reference is dead code (missing module); ``qrnn=True`` raises.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


def _mask(x: torch.Tensor, size, p: float) -> torch.Tensor:
    return x.new_empty(size).bernoulli_(1 - p).div_(1 - p)


class LockedDropout(nn.Module):
    """One dropout mask per (batch, feature), shared over the sequence axis (dim 0)."""

    def __init__(self, p: float = 0.5):
        super().__init__()
        self.p = p

    def forward(self, x):
        if not self.training or self.p == 0:
            return x
        return x * _mask(x, (1, x.size(1), x.size(2)), self.p)


class EmbeddingRowDropout(nn.Module):
    """Embedding lookup that drops whole vocabulary rows in training (shares ``emb``)."""

    def __init__(self, emb: nn.Embedding, p: float):
        super().__init__()
        self.emb, self.p = emb, p

    def forward(self, idx):
        w = self.emb.weight
        if self.training and self.p:
            w = w * _mask(w, (w.size(0), 1), self.p)
        pad = self.emb.padding_idx if self.emb.padding_idx is not None else -1
        return F.embedding(idx, w, pad)


class DropConnectLSTM(nn.Module):
    """Single-layer LSTM whose hidden-to-hidden matrix is DropConnect-ed in training.

    Keeps the raw matrix as ``weight_hh_l0_raw`` (a Parameter) next to ``module`` (the
    ``nn.LSTM``), giving the checkpoint keys of the reference. ``bidir``: a bidirectional
    layer of ``n_out // 2`` units per direction (reference awd_lstm.py:57,69-70); as in the
    reference's ``WeightDropout(rnn, weight_p)`` only the forward direction's ``weight_hh_l0``
    is DropConnect-ed (``_reverse`` weights are plain LSTM parameters).
    """

    def __init__(self, n_in: int, n_out: int, p: float, bidir: bool = False):
        super().__init__()
        self.ndir = 2 if bidir else 1
        self.module = nn.LSTM(n_in, n_out // self.ndir, 1, bidirectional=bidir)
        self.p = p
        self.weight_hh_l0_raw = nn.Parameter(self.module.weight_hh_l0.detach().clone())

    def sync_from_module(self):
        with torch.no_grad():
            self.weight_hh_l0_raw.copy_(self.module.weight_hh_l0)

    def forward(self, x, hc):
        w_hh = F.dropout(self.weight_hh_l0_raw, self.p, self.training) if self.training else self.module.weight_hh_l0
        m = self.module
        ws = [m.weight_ih_l0, w_hh, m.bias_ih_l0, m.bias_hh_l0]
        if self.ndir == 2:
            ws += [m.weight_ih_l0_reverse, m.weight_hh_l0_reverse, m.bias_ih_l0_reverse, m.bias_hh_l0_reverse]
        out, h, c = torch._VF.lstm(x, hc, ws, True, 1, 0.0, self.training, self.ndir == 2, False)
        return out, (h, c)


class RNNCore(nn.Module):
    def __init__(self, vocab_sz, emb_sz, n_hid, n_layers, pad_token, bidir=False, hidden_p=0.2, input_p=0.6,
                 embed_p=0.1, weight_p=0.5, qrnn=False):
        super().__init__()
        if qrnn:
            raise NotImplementedError("QRNN is dead code in the reference (missing module); not supported")
        self.ndir = 2 if bidir else 1
        self.bs = 1
        self.emb_sz, self.n_hid, self.n_layers = emb_sz, n_hid, n_layers
        self.encoder = nn.Embedding(vocab_sz, emb_sz, padding_idx=pad_token)
        self.encoder_dp = EmbeddingRowDropout(self.encoder, embed_p)
        dims = [emb_sz] + [n_hid] * (n_layers - 1) + [emb_sz]
        self.rnns = nn.ModuleList([DropConnectLSTM(dims[i], dims[i + 1], weight_p, bidir) for i in range(n_layers)])
        self.encoder.weight.data.uniform_(-0.1, 0.1)
        self.input_dp = LockedDropout(input_p)
        self.hidden_dps = nn.ModuleList([LockedDropout(hidden_p) for _ in range(n_layers)])
        self.hidden = None

    def layer_dims(self):
        return [(r.module.input_size, r.module.hidden_size) for r in self.rnns]

    def reset(self):
        p = self.encoder.weight
        self.hidden = [(p.new_zeros(r.ndir, self.bs, r.module.hidden_size),
                        p.new_zeros(r.ndir, self.bs, r.module.hidden_size)) for r in self.rnns]

    def forward(self, inp):
        sl, bs = inp.shape
        if bs != self.bs or self.hidden is None:
            self.bs = bs
            self.reset()
        x = self.input_dp(self.encoder_dp(inp))
        new_hidden, raw_outputs, outputs = [], [], []
        for l, (rnn, dp) in enumerate(zip(self.rnns, self.hidden_dps)):
            x, hc = rnn(x, self.hidden[l])
            new_hidden.append(hc)
            raw_outputs.append(x)
            if l != self.n_layers - 1:
                x = dp(x)
            outputs.append(x)
        self.hidden = [(h.detach(), c.detach()) for (h, c) in new_hidden]
        return raw_outputs, outputs


class LinearDecoder(nn.Module):
    def __init__(self, n_out, n_hid, output_p, tie_encoder=None, bias=True):
        super().__init__()
        self.decoder = nn.Linear(n_hid, n_out, bias=bias)
        self.decoder.weight.data.uniform_(-0.1, 0.1)
        if bias:
            self.decoder.bias.data.zero_()
        if tie_encoder is not None:
            self.decoder.weight = tie_encoder.weight
        self.output_dp = LockedDropout(output_p)

    def forward(self, inp):
        raw_outputs, outputs = inp
        o = self.output_dp(outputs[-1])
        return self.decoder(o.reshape(-1, o.size(-1))), raw_outputs, outputs


class LanguageModel(nn.Sequential):
    """``[0]`` = RNNCore, ``[1]`` = LinearDecoder; ``reset()`` forwards to children."""

    def reset(self):
        for c in self.children():
            if hasattr(c, "reset"):
                c.reset()

    def load_state_dict(self, sd, strict: bool = True, assign: bool = False):
        sd = dict(sd)
        # effective W_hh is the checkpoint's module.weight_hh_l0 (else _raw)
        for l in range(len(self[0].rnns)):
            raw, mod = f"0.rnns.{l}.weight_hh_l0_raw", f"0.rnns.{l}.module.weight_hh_l0"
            if mod in sd:
                sd[raw] = sd[mod]
            elif raw in sd:
                sd[mod] = sd[raw]
        enc = "0.encoder.weight"
        for alias in ("0.encoder_dp.emb.weight", "1.decoder.weight"):
            if alias not in sd and enc in sd:
                sd[alias] = sd[enc]
        res = super().load_state_dict(sd, strict=strict, assign=assign)
        self.reset()
        return res

    @property
    def bs(self):
        return self[0].bs


def get_language_model(vocab_sz: int, emb_sz: int, n_hid: int, n_layers: int, pad_token: int,
                       tie_weights: bool = True, qrnn: bool = False, bias: bool = True, bidir: bool = False,
                       output_p: float = 0.4, hidden_p: float = 0.2, input_p: float = 0.6, embed_p: float = 0.1,
                       weight_p: float = 0.5) -> LanguageModel:
    core = RNNCore(vocab_sz, emb_sz, n_hid, n_layers, pad_token, bidir, hidden_p, input_p, embed_p, weight_p, qrnn)
    dec = LinearDecoder(vocab_sz, emb_sz, output_p, core.encoder if tie_weights else None, bias)
    m = LanguageModel(core, dec)
    m.reset()
    return m


# the reference's serving hyper-parameters (main.py:95-96)
REFERENCE_DPS = (0.25, 0.1, 0.2, 0.02, 0.15)  # input, output, weight, embed, hidden


def reference_lm(vocab_sz: int) -> LanguageModel:
    i, o, w, e, h = REFERENCE_DPS
    return get_language_model(vocab_sz, emb_sz=1000, n_hid=1150, n_layers=3, pad_token=1, input_p=i,
                              output_p=o, weight_p=w, embed_p=e, hidden_p=h, tie_weights=True, bias=True,
                              qrnn=False)
