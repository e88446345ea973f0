"""Pure-PyTorch interpreter of a lowered :class:`Graph` (fp32 oracle of the native program).

It executes exactly the nodes/packed weights the native program will run, with torch ops,
so the lowering (BN folding, weight packing/padding, NHWC layout, residual wiring, fork/join
ordering) is checked on CPU against the eager model, and the GPU kernels are checked against
this node-by-node. ``bf16_acts=True`` rounds every stored activation to bf16 like the device
does, which isolates accumulation-order error from storage rounding.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .graph import Graph


def _conv_ref(x_nhwc, pc, res=None, act="relu", out_f32=False):
    w = pc.dense().reshape(pc.cout, pc.r, pc.s, pc.cin).permute(0, 3, 1, 2)
    y = F.conv2d(x_nhwc.permute(0, 3, 1, 2).float(), w, pc.bias.float(), stride=pc.stride, padding=pc.pad)
    y = y.permute(0, 2, 3, 1)
    if res is not None:
        y = y + res.float()
    if act == "relu":
        y = torch.relu(y)
    elif act == "gelu":
        y = F.gelu(y)
    elif act == "tanh":
        y = torch.tanh(y)
    return y


def run_graph_reference(g: Graph, params: dict, inputs: list, bf16_acts: bool = True) -> dict:
    vals: dict[int, torch.Tensor] = {}
    for tid, x in zip(g.inputs, inputs):
        vals[tid] = x

    def store(tid, v):
        spec = g.tensors[tid]
        if bf16_acts and spec.dtype == torch.bfloat16:
            v = v.to(torch.bfloat16).float()
        vals[tid] = v.reshape(spec.shape)

    for n in g.nodes:
        k = n.kind
        if k in ("fork", "join"):
            continue
        if k == "preprocess":
            src = vals[n.inputs[0]]
            cpad = g.shape(n.outputs[0])[-1]
            if src.dtype == torch.uint8:
                x = src.float() / 255.0
            else:
                x = src.float().permute(0, 2, 3, 1)
            if n.attrs.get("mean") is not None:
                x = (x - torch.tensor(n.attrs["mean"])) / torch.tensor(n.attrs["std"])
            store(n.outputs[0], F.pad(x, (0, cpad - x.shape[-1])))
        elif k == "patchify":
            x = vals[n.inputs[0]].float()
            if n.attrs.get("mean") is not None:
                x = (x - torch.tensor(n.attrs["mean"])[:, None, None]) / torch.tensor(n.attrs["std"])[:, None, None]
            P = n.attrs["patch"]
            nb, c, h, w = x.shape
            x = x.reshape(nb, c, h // P, P, w // P, P).permute(0, 2, 4, 1, 3, 5)  # n, py, px, c, ky, kx
            store(n.outputs[0], x.reshape(nb * (h // P) * (w // P), c * P * P))
        elif k == "conv":
            pc = params[n.attrs["w"]]
            res = vals[n.inputs[1]] if len(n.inputs) > 1 else None
            y = _conv_ref(vals[n.inputs[0]], pc, res, n.attrs.get("act", "relu"))
            store(n.outputs[0], y.reshape(g.shape(n.outputs[0])))
        elif k == "maxpool":
            a = n.attrs
            x = vals[n.inputs[0]].permute(0, 3, 1, 2)
            y = F.max_pool2d(x, a["k"], a["stride"], a["pad"]).permute(0, 2, 3, 1)
            store(n.outputs[0], y)
        elif k == "avgpool":
            x = vals[n.inputs[0]]
            store(n.outputs[0], x.float().mean(dim=(1, 2), keepdim=True))
        elif k == "gemm":
            pc = params[n.attrs["w"]]
            x = vals[n.inputs[0]].float().reshape(-1)
            rows, ldx = n.attrs["rows"], n.attrs.get("ldx") or g.shape(n.inputs[0])[-1]
            xm = torch.stack([x[r * ldx: r * ldx + pc.K] for r in range(rows)])
            w = pc.dense() if not hasattr(pc, "dequant") else pc.dequant()
            a = n.attrs
            y = xm @ w.t()
            if a.get("ln_in"):  # folded LayerNorm of the raw input (stats taken from the input itself)
                eps = params[a["ln_in"][0]].eps
                mu, var = xm.mean(1, keepdim=True), xm.var(1, unbiased=False, keepdim=True)
                y = torch.rsqrt(var + eps) * (y - mu * params[a["w"] + ".c1"].float()[None, :])
            y = y + pc.bias.float()
            if a.get("has_res", len(n.inputs) > 1):
                r = vals[n.inputs[1]].float().reshape(rows, -1)
                if a.get("res_ln"):
                    npar = params[a["res_ln"][0]]
                    r = F.layer_norm(r, (r.shape[-1],), npar.gamma.float(), npar.beta.float(), npar.eps)
                y = y + r
            act = a.get("act", "none")
            y = torch.relu(y) if act == "relu" else F.gelu(y) if act == "gelu" else torch.tanh(y) if act == "tanh" else y
            if a.get("stats_out") is not None:  # the oracle's consumers recompute statistics themselves
                store(n.outputs[0], y)
                vals[a["stats_out"]] = torch.zeros(g.shape(a["stats_out"]))
            elif len(n.outputs) == 2:  # MX8 output
                from ..ops.fp8 import quant_mx_ref
                vals[n.outputs[0]], vals[n.outputs[1]] = quant_mx_ref(y)
            else:
                store(n.outputs[0], y)
        elif k == "quant":
            from ..ops.fp8 import quant_rows_ref
            deq, s = quant_rows_ref(vals[n.inputs[0]])
            vals[n.outputs[0]] = deq  # the oracle carries the dequantised values
            vals[n.outputs[1]] = s
        elif k == "gemm_fp8":
            pw = params[n.attrs["w"]]
            y = vals[n.inputs[0]].float() @ pw.dequant().t() + pw.bias.float()
            if len(n.inputs) > 2:
                y = y + vals[n.inputs[2]].float()
            act = n.attrs.get("act", "none")
            y = torch.relu(y) if act == "relu" else F.gelu(y) if act == "gelu" else torch.tanh(y) if act == "tanh" else y
            if len(n.outputs) == 2:  # MX8 output
                from ..ops.fp8 import quant_mx_ref
                vals[n.outputs[0]], vals[n.outputs[1]] = quant_mx_ref(y)
            else:
                store(n.outputs[0], y)
        elif k == "layernorm":
            npar = params[n.attrs["p"]]
            rows = n.attrs["rows"]
            D = g.shape(n.outputs[0])[-1]
            ldx = n.attrs.get("ldx") or D
            x = vals[n.inputs[0]].float().reshape(-1)
            xm = torch.stack([x[r * ldx: r * ldx + D] for r in range(rows)])
            if len(n.inputs) > 1:
                xm = xm + vals[n.inputs[1]].float().reshape(rows, D)
            y = F.layer_norm(xm, (D,), npar.gamma.float(), npar.beta.float(), npar.eps)
            outs = list(n.outputs)
            if g.tensors[outs[0]].dtype != torch.uint8:
                store(outs.pop(0), y)
            if outs:  # fused fp8 quantisation
                from ..ops.fp8 import quant_rows_ref
                deq, s = quant_rows_ref(y.to(torch.bfloat16))
                vals[outs[0]], vals[outs[1]] = deq, s
        elif k == "attention":
            a = n.attrs
            mask = vals[n.inputs[1]] if len(n.inputs) > 1 else None
            from ..ops.transformer import attention_ref
            y = attention_ref(vals[n.inputs[0]], a["B"], a["L"], a["heads"], mask)
            if len(n.outputs) == 2:  # MX8 output: the oracle carries the dequantised values
                from ..ops.fp8 import quant_mx_ref
                vals[n.outputs[0]], vals[n.outputs[1]] = quant_mx_ref(y.to(torch.bfloat16))
            else:
                store(n.outputs[0], y)
        elif k == "embed_ln":
            from ..ops.transformer import embed_ref
            tab, ln = params[n.attrs["emb"]], params[n.attrs["ln"]]
            store(n.outputs[0], embed_ref(vals[n.inputs[0]], vals[n.inputs[1]], tab, ln, n.attrs["L"]))
        elif k == "pool_fc":
            from ..ops.vision import pool_fc_ref
            x = vals[n.inputs[0]].float().reshape(g.shape(n.inputs[0]))
            store(n.outputs[0], pool_fc_ref(x, params[n.attrs["w"]]))
        elif k == "softmax":
            from ..ops.transformer import softmax_ref
            x = vals[n.inputs[0]].float().reshape(g.shape(n.inputs[0])[0], -1)
            store(n.outputs[0], softmax_ref(x, n.attrs.get("D"), float(n.attrs.get("scale", 1.0))))
        elif k == "vit_tokens":
            a = n.attrs
            D = g.shape(n.outputs[0])[-1]
            pt = vals[n.inputs[0]].float().reshape(a["B"], a["np"], D)
            cls = params[a["cls"]].float().reshape(1, 1, D).expand(a["B"], 1, D)
            store(n.outputs[0], torch.cat([cls, pt], 1) + params[a["pos"]].float().reshape(1, a["np"] + 1, D))
        else:
            raise NotImplementedError(k)
    return vals
