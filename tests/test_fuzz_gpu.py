"""Hypothesis shape fuzzing of the hand-written kernels vs fp32 PyTorch (SURVEY.md §4.2
T-kernel-gpu): random GEMM (M, N, K) incl. ragged tails on every path the dispatcher picks,
random convolution geometries, LayerNorm widths and attention lengths."""
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from hipzap.ops import conv as C
from hipzap.ops import transformer as T

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
FUZZ = settings(max_examples=25, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])


def _rel(a, b):
    return ((a.float().cpu() - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


@FUZZ
@given(M=st.integers(1, 700), N=st.integers(1, 96).map(lambda n: 4 * n), K=st.integers(1, 48).map(lambda k: 32 * k),
       act=st.sampled_from(["none", "relu", "gelu", "tanh"]), res=st.booleans(), seed=st.integers(0, 2**16))
def test_gemm_shapes(M, N, K, act, res, seed):
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(N, K, generator=g) * K ** -0.5
    b = torch.randn(N, generator=g)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    r = torch.randn(M, N, generator=g).to(torch.bfloat16) if res else None
    pc = C.pack_linear(w, b).to(DEV)
    y = C.linear(x.to(DEV), pc, residual=None if r is None else r.to(DEV), act=act)
    ref = x.float() @ w.to(torch.bfloat16).float().t() + b + (r.float() if res else 0)
    ref = {"gelu": torch.nn.functional.gelu, "relu": torch.relu, "tanh": torch.tanh}.get(act, lambda t: t)(ref)
    assert _rel(y, ref) < 2e-2


@FUZZ
@given(n=st.integers(1, 2), cin=st.sampled_from([8, 16, 32, 64, 96, 128]), h=st.integers(3, 20),
       cout=st.sampled_from([16, 32, 48, 64, 128]), k=st.sampled_from([1, 3]), stride=st.sampled_from([1, 2]),
       res=st.booleans(), seed=st.integers(0, 2**16))
def test_conv_shapes(n, cin, h, cout, k, stride, res, seed):
    pad = k // 2
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, cin, h, h, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    pc = C.pack_conv(w, b, None, stride, pad)
    p = (h + 2 * pad - k) // stride + 1
    r = torch.randn(n, cout, p, p, generator=g) if res else None
    xb = x.to(torch.bfloat16).float()
    wref = pc.dense().reshape(cout, k, k, pc.cin)[..., :cin].permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(xb, wref, pc.bias, stride=stride, padding=pad)
    if r is not None:
        ref = ref + r.to(torch.bfloat16).float()
    ref = torch.relu(ref)
    x_nhwc = torch.nn.functional.pad(xb.permute(0, 2, 3, 1), (0, pc.cin - cin)).to(torch.bfloat16)
    r_nhwc = None if r is None else r.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(DEV)
    out = C.conv2d_nhwc(x_nhwc.contiguous().to(DEV), pc.to(DEV), r_nhwc, act="relu")
    assert _rel(out.permute(0, 3, 1, 2), ref) < 2e-2


@FUZZ
@given(rows=st.integers(1, 300), D=st.sampled_from([64, 128, 256, 384, 512, 768, 1024]), res=st.booleans(),
       seed=st.integers(0, 2**16))
def test_layernorm_shapes(rows, D, res, seed):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(rows, D, generator=g) * 3).to(torch.bfloat16)
    r = torch.randn(rows, D, generator=g).to(torch.bfloat16) if res else None
    npar = T.NormParams(torch.randn(D, generator=g), torch.randn(D, generator=g), 1e-5)
    y = T.layernorm(x.to(DEV), npar.to(DEV), residual=None if r is None else r.to(DEV))
    assert _rel(y, T.layernorm_ref(x, npar, r)) < 2e-2


@FUZZ
@given(B=st.integers(1, 3), L=st.integers(1, 256), heads=st.integers(1, 4), masked=st.booleans(),
       seed=st.integers(0, 2**16))
def test_attention_lengths(B, L, heads, masked, seed):
    g = torch.Generator().manual_seed(seed)
    qkv = torch.randn(B * L, 3 * heads * 64, generator=g).to(torch.bfloat16)
    mask = None
    if masked:
        keep = torch.rand(B, L, generator=g) > 0.3
        keep[:, 0] = True
        mask = torch.where(keep, 0.0, -10000.0).float()
    out = T.attention(qkv.to(DEV), B, L, heads, None if mask is None else mask.to(DEV))
    assert _rel(out, T.attention_ref(qkv, B, L, heads, mask)) < 2e-2
