"""FP8 (OCP e4m3fn) quantisation + fp8 MFMA GEMM on MI355X."""
import pytest
import torch

from hipzap.engine.engine import Engine
from hipzap.models import vit
from hipzap.ops import conv as C
from hipzap.ops import fp8 as F8

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _need_exp(cfg):
    """cfg 34-36 (ping-pong) and 43-47 (256-row MX pipelines) exist only in the HZ_EXPERIMENTS library."""
    from hipzap import _native as N
    if cfg in F8.MX_EXPERIMENTS and not N.experiments():
        pytest.skip("measured-negative MX pipeline: build with python -m hipzap.build --experiments")


def test_quant_rows_is_ocp_e4m3fn():
    g = torch.Generator().manual_seed(0)
    x = (torch.randn(37, 768, generator=g) * 3).to(torch.bfloat16)
    q, s = F8.quant_rows(x.to(DEV))
    s_ref = x.float().abs().amax(1).clamp_min(1e-12) / 448.0
    assert torch.allclose(s.cpu(), s_ref, rtol=1e-6)
    ref_bits = (x.float() / s_ref[:, None]).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    mism = (q.cpu() != ref_bits).float().mean().item()
    assert mism < 1e-3, mism  # identical encoding (OCP, not FNUZ); rounding ties may differ


@pytest.mark.parametrize("M,N,K", [(1576, 2304, 768), (8, 1000, 768), (197, 768, 3072)])
def test_gemm_fp8(M, N, K):
    g = torch.Generator().manual_seed(1)
    w = torch.randn(N, K, generator=g) * 0.05
    b = torch.randn(N, generator=g)
    x = torch.randn(M, K, generator=g).to(torch.bfloat16)
    r = torch.randn(M, N, generator=g).to(torch.bfloat16)
    pw = F8.quantize_linear(C.pack_linear(w, b))
    pwd = F8.PackedFp8(pw.w8.to(DEV), pw.sw.to(DEV), pw.bias.to(DEV), pw.cin, pw.cout)
    x8, sx = F8.quant_rows(x.to(DEV))
    y = F8.gemm_fp8(x8, sx, pwd, residual=r.to(DEV), act="gelu")
    xd, _ = F8.quant_rows_ref(x)
    ref = torch.nn.functional.gelu(xd @ pw.dequant().t() + b + r.float())
    rel = ((y.float().cpu() - ref).abs().max() / ref.abs().max()).item()
    assert rel < 2e-2, rel


def test_vit_fp8_engine_vs_hf():
    """fp8 against the bf16 engine on the same weights (per-row cosine, top-1) and HF fp32."""
    torch.manual_seed(0)
    m = vit.make_model(num_labels=1000)
    sd = m.state_dict()
    eng = Engine.from_state_dict("vit-b16-fp8", sd, DEV, batch=4)
    bf = Engine.from_state_dict("vit-b16", sd, DEV, batch=4)
    x = torch.randn(4, 3, 224, 224)
    out, ref16 = eng.infer(x), bf.infer(x)
    with torch.no_grad():
        ref = m(pixel_values=x).logits
    cos16 = torch.nn.functional.cosine_similarity(out, ref16, dim=1)
    assert cos16.min() > 0.99, cos16
    assert torch.equal(out.argmax(1), ref16.argmax(1))
    # measured on MI355X (scripts/check_vit_fp8_err.py, same seed) vs HF fp32: cos 0.993, top-1
    # equal (bf16 engine 0.99993); e4m3 weights + per-row e4m3 activations through 12 layers
    cos = torch.nn.functional.cosine_similarity(out, ref, dim=1)
    assert cos.min() > 0.99, cos
    assert torch.equal(out.argmax(1), ref.argmax(1))


def test_layernorm_fused_fp8_quant():
    """LayerNorm + per-row fp8 quantisation in one kernel == LN then quant_rows."""
    from hipzap.ops import transformer as T
    g = torch.Generator().manual_seed(4)
    x = torch.randn(300, 768, generator=g).to(torch.bfloat16)
    r = torch.randn(300, 768, generator=g).to(torch.bfloat16)
    npar = T.NormParams(torch.randn(768, generator=g), torch.randn(768, generator=g), 1e-6)
    x8, sx, y = T.layernorm_q8(x.to(DEV), npar.to(DEV), residual=r.to(DEV), keep_bf16=True)
    ref = T.layernorm_ref(x, npar, r)
    assert ((y.float().cpu() - ref).abs().max() / ref.abs().max()).item() < 2e-2
    deq_ref, s_ref = F8.quant_rows_ref(ref)
    assert torch.allclose(sx.cpu(), s_ref, rtol=2e-2)
    deq = x8.cpu().view(torch.float8_e4m3fn).float() * sx.cpu()[:, None]
    assert ((deq - deq_ref).abs().max() / deq_ref.abs().max()).item() < 5e-2


def _probe_f8f6f4(layout: int, A: torch.Tensor, Bt: torch.Tensor) -> torch.Tensor:
    import ctypes
    from hipzap import _native as N
    ab = torch.cat([A.to(torch.float8_e4m3fn).view(torch.uint8).reshape(-1),
                    Bt.to(torch.float8_e4m3fn).view(torch.uint8).reshape(-1)]).to(DEV)
    c = torch.zeros(16, 16, device=DEV)
    N.check(N.lib().hz_diag_launch(2, layout, 64, ctypes.c_void_p(ab.data_ptr()), ctypes.c_void_p(c.data_ptr()), 0,
                                   N.stream_ptr()), "probe")
    torch.cuda.synchronize()
    return c.cpu()


def test_mfma_f8f6f4_operand_layout():
    """What csrc/fp8.hip's MX GEMM relies on (unit block scales): the hardware applies the SAME
    lane->k permutation to A and B, so any map used consistently for both operands (weights
    MX-packed, activations gathered with the same map) yields the exact dot product, and mixing
    two different maps does not (exact small integers, so equality is exact)."""
    g = torch.Generator().manual_seed(7)
    A = torch.randint(-3, 4, (16, 128), generator=g).float()
    Bt = torch.randint(-3, 4, (16, 128), generator=g).float()
    ref = A @ Bt.t()
    assert torch.equal(_probe_f8f6f4(0, A, Bt), ref)   # both operands: 32 consecutive k per lane
    assert torch.equal(_probe_f8f6f4(3, A, Bt), ref)   # both operands: 4 blocks of the 16x16x32 map
    assert not torch.equal(_probe_f8f6f4(1, A, Bt), ref)  # inconsistent maps are detected


def _mx_encode(x: torch.Tensor):
    """Host MX8 encoding (quant_mx_ref rule): e4m3 bytes + E8M0 bytes [rows, cols/32]."""
    deq, e = F8.quant_mx_ref(x)
    sc = torch.ldexp(torch.ones_like(e, dtype=torch.float32), e).repeat_interleave(32, 1)
    q8 = (deq / sc).to(torch.float8_e4m3fn).view(torch.uint8)
    return q8, (e + 127).to(torch.uint8), deq


def _mx_decode(q8: torch.Tensor, s8: torch.Tensor) -> torch.Tensor:
    sc = torch.ldexp(torch.ones(s8.shape), s8.long() - 127).repeat_interleave(32, 1)
    return q8.view(torch.float8_e4m3fn).float() * sc


@pytest.mark.parametrize("cfg", [16, 19, 21, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 40, 41, 42])
@pytest.mark.parametrize("mx_in,mx_out", [(True, False), (False, True), (True, True)])
def test_gemm_mx8_activations(cfg, mx_in, mx_out):
    """MX8 (e4m3 + E8M0 per 32 k) activations into the block-scaled MFMA, and MX8 output from
    the epilogue, vs the fp32 oracle of the same quantisation."""
    _need_exp(cfg)
    import ctypes
    from hipzap import _native as N
    g = torch.Generator().manual_seed(9)
    M, Nn, K = 200, 768, 512
    w = torch.randn(Nn, K, generator=g) * 0.05
    b = torch.randn(Nn, generator=g)
    x = torch.randn(M, K, generator=g) * torch.linspace(0.1, 8, K)  # per-block dynamic ranges differ
    pw = F8.quantize_linear(C.pack_linear(w, b))
    pwd = F8.PackedFp8(pw.w8.to(DEV), pw.sw.to(DEV), pw.bias.to(DEV), pw.cin, pw.cout, pw.w8mx.to(DEV))
    if mx_in:
        q8, s8, xd = _mx_encode(x)
        x8, xs, sx = q8.to(DEV), s8.to(DEV), None
    else:
        x8, sx = F8.quant_rows(x.to(torch.bfloat16).to(DEV))
        xd, _ = F8.quant_rows_ref(x.to(torch.bfloat16))
        xs = None
    ref = torch.nn.functional.gelu(xd @ pw.dequant().t() + b)
    out = torch.empty(M, Nn, device=DEV, dtype=torch.bfloat16)
    o8 = torch.zeros(M, Nn, dtype=torch.uint8, device=DEV)
    os8 = torch.zeros(M, Nn // 32, dtype=torch.uint8, device=DEV)
    prm = F8.gemm_params(x8.data_ptr(), N.ptr(sx), pwd, M, 0 if mx_out else out.data_ptr(), 0, "gelu", False, cfg,
                         1, xs_ptr=N.ptr(xs), out8_ptr=o8.data_ptr() if mx_out else 0,
                         os8_ptr=os8.data_ptr() if mx_out else 0)
    N.check(N.lib().hz_launch_kernel(F8.K_GEMM_FP8, ctypes.byref(prm), N.stream_ptr()), "gemm mx8")
    torch.cuda.synchronize()
    if mx_out:
        got = _mx_decode(o8.cpu(), os8.cpu())
        ref_q, _ = F8.quant_mx_ref(ref)
        assert ((got - ref_q).abs().max() / ref_q.abs().max()).item() < 0.1  # <= one e4m3 step
    else:
        assert ((out.float().cpu() - ref).abs().max() / ref.abs().max()).item() < 2e-2


@pytest.mark.parametrize("cfg", [33, 40, 41, 42])
@pytest.mark.parametrize("mx_in,mx_out", [(False, False), (True, True)])
def test_gemm_mx256_bitwise_vs_128(cfg, mx_in, mx_out):
    """The plain 256x256 MX tile (cfg 33) sums every output over the same k-steps in the same order
    with the same instruction and epilogue as the 8-wave 128x128 kernel (cfg 24): results are
    BITWISE equal, over several row tiles (one partial) and column tiles, bf16 or MX8 output.
    (The 256-row / ping-pong variants 34-36 and 43-47 were removed in round 5; their bitwise tests
    with them.)"""
    _need_exp(cfg)
    import ctypes
    from hipzap import _native as N
    g = torch.Generator().manual_seed(11)
    M, Nn, K = 700, 768, 1024
    w = torch.randn(Nn, K, generator=g) * 0.05
    b = torch.randn(Nn, generator=g)
    x = torch.randn(M, K, generator=g) * torch.linspace(0.1, 8, K)
    pw = F8.quantize_linear(C.pack_linear(w, b))
    pwd = F8.PackedFp8(pw.w8.to(DEV), pw.sw.to(DEV), pw.bias.to(DEV), pw.cin, pw.cout, pw.w8mx.to(DEV))
    if mx_in:
        q8, s8, _ = _mx_encode(x)
        x8, xs, sx = q8.to(DEV), s8.to(DEV), None
    else:
        x8, sx = F8.quant_rows(x.to(torch.bfloat16).to(DEV))
        xs = None
    outs = []
    for c in (24, cfg):
        out = torch.full((M, Nn), 7.0, device=DEV, dtype=torch.bfloat16)
        o8 = torch.zeros(M, Nn, dtype=torch.uint8, device=DEV)
        os8 = torch.zeros(M, Nn // 32, dtype=torch.uint8, device=DEV)
        prm = F8.gemm_params(x8.data_ptr(), N.ptr(sx), pwd, M, 0 if mx_out else out.data_ptr(), 0, "gelu", False, c,
                             1, xs_ptr=N.ptr(xs), out8_ptr=o8.data_ptr() if mx_out else 0,
                             os8_ptr=os8.data_ptr() if mx_out else 0)
        N.check(N.lib().hz_launch_kernel(F8.K_GEMM_FP8, ctypes.byref(prm), N.stream_ptr()), f"gemm cfg {c}")
        torch.cuda.synchronize()
        outs.append((o8.cpu(), os8.cpu()) if mx_out else (out.cpu(),))
    for a, b_ in zip(*outs):
        assert torch.equal(a, b_), f"cfg {cfg} differs from cfg 24"
    if not mx_out:
        assert not (outs[1][0] == 7.0).all(-1).any(), "rows left unwritten"


def test_attention_mx8_output():
    from hipzap.ops import transformer as T
    import ctypes
    from hipzap import _native as N
    g = torch.Generator().manual_seed(10)
    B, L, H = 2, 197, 12
    qkv = torch.randn(B * L, 3 * H * 64, generator=g).to(torch.bfloat16)
    ref = T.attention_ref(qkv, B, L, H, None)
    o8 = torch.zeros(B * L, H * 64, dtype=torch.uint8, device=DEV)
    os8 = torch.zeros(B * L, H * 2, dtype=torch.uint8, device=DEV)
    q = qkv.to(DEV)
    D = H * 64
    prm = T.AttentionParams(q.data_ptr(), 0, 0, B, L, H, 64, q.stride(0), D, 2 * D, D, 0.125, o8.data_ptr(),
                            os8.data_ptr())
    N.check(N.lib().hz_launch_kernel(T.K_ATTENTION, ctypes.byref(prm), N.stream_ptr()), "attention mx8")
    torch.cuda.synchronize()
    got = _mx_decode(o8.cpu(), os8.cpu())
    ref_q, _ = F8.quant_mx_ref(ref.float())
    assert ((got - ref_q).abs().max() / ref_q.abs().max()).item() < 0.1  # <= one e4m3 step


def _probe_scales(A, Bt, sa, sb):
    import ctypes
    from hipzap import _native as N
    buf = torch.cat([A.to(torch.float8_e4m3fn).view(torch.uint8).reshape(-1),
                     Bt.to(torch.float8_e4m3fn).view(torch.uint8).reshape(-1),
                     torch.tensor(sa, dtype=torch.int32).view(torch.uint8),
                     torch.tensor(sb, dtype=torch.int32).view(torch.uint8)]).to(DEV)
    c = torch.zeros(16, 16, device=DEV)
    N.check(N.lib().hz_diag_launch(3, 1, 64, ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(c.data_ptr()), 0,
                                   N.stream_ptr()), "probe scale")
    torch.cuda.synchronize()
    return c.cpu()


def test_mfma_block_scale_lane_map():
    """Which lane's scale byte scales which (row/column, 32-k block) of the f8f6f4 MFMA:
    csrc/fp8.hip feeds the activation (B) scale of token l&15, k-block l>>4 from lane l."""
    ones = torch.ones(16, 128)
    found = {}
    for operand in ("a", "b"):
        for lane in (0, 1, 17, 33, 50):
            sa, sb = [127] * 64, [127] * 64
            (sa if operand == "a" else sb)[lane] = 129  # x4 on one lane's block
            d = _probe_scales(ones, ones, sa, sb)
            diff = (d != 128).nonzero().tolist()
            found[(operand, lane)] = diff
    # expected (H1): lane l scales A row l&15 (resp. B column l&15) for k-block l>>4:
    # one 32-k block x4 -> that row/column sums 3*32 + 4*32 = 224
    for (operand, lane), diff in found.items():
        rows = sorted({r for r, _ in diff})
        cols = sorted({c for _, c in diff})
        if operand == "a":
            assert rows == [lane & 15] and len(cols) == 16, (operand, lane, diff[:4], found)
        else:
            assert cols == [lane & 15] and len(rows) == 16, (operand, lane, diff[:4], found)


def _probe_raw(a_regs, b_regs, sa, sb):
    """a_regs/b_regs: [64 lanes, 32] fp32 values placed verbatim in the operand registers."""
    import ctypes
    from hipzap import _native as N
    buf = torch.cat([a_regs.to(torch.float8_e4m3fn).view(torch.uint8).reshape(-1),
                     b_regs.to(torch.float8_e4m3fn).view(torch.uint8).reshape(-1),
                     torch.tensor(sa, dtype=torch.int32).view(torch.uint8),
                     torch.tensor(sb, dtype=torch.int32).view(torch.uint8)]).to(DEV)
    c = torch.zeros(16, 16, device=DEV)
    N.check(N.lib().hz_diag_launch(4, 1, 64, ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(c.data_ptr()), 0,
                                   N.stream_ptr()), "probe scale raw")
    torch.cuda.synchronize()
    return c.cpu()


def mfma_scale_kblock_map() -> dict:
    """{(lane group g, register byte j): lane group whose B-scale applies to that byte}.
    A = ones; B = one nonzero register byte (g, j) in every lane of group g; B scales 2^h for
    lane group h -> D = 2^(governing group)."""
    out = {}
    sa = [127] * 64
    sb = [127 + (lane >> 4) for lane in range(64)]
    a = torch.ones(64, 32)
    for g in range(4):
        for j in range(32):
            b = torch.zeros(64, 32)
            b[16 * g: 16 * g + 16, j] = 1.0
            d = _probe_raw(a, b, sa, sb)
            v = d[0, 0].item()
            assert torch.all(d == v), d
            out[(g, j)] = int(round(torch.log2(torch.tensor(v)).item()))
    return out


def test_mfma_block_scale_kblock_map():
    """The hardware K order the block scales follow: register byte j of lane group g is
    k = 64*(j//16) + 16*g + j%16, i.e. in 32-k block 2*(j//16) + g//2, and lane group b's scale
    byte scales block b. csrc/fp8.hip (gemm_mx_kernel) and ops/fp8.py (mx_pack) place the data
    in this order. (Unscaled MFMA results cannot see this: any K permutation shared by A and B
    gives the same dot product, which is why the operand-layout probe above passes either way.)"""
    m = mfma_scale_kblock_map()
    assert all(m[(g, j)] == 2 * (j // 16) + g // 2 for g in range(4) for j in range(32)), m


@pytest.mark.parametrize("cfg", [40, 41, 42])
@pytest.mark.parametrize("K", [128, 256, 384, 3072])
def test_gemm_mx_role_split_short_and_long_k(cfg, K):
    """The role-split kernels' ring at fewer k-steps than stages (K 128 / 256 / 384: the loaders'
    drain publishes the last stages) and at many (K 3072: 24 rounds of every slot): bitwise cfg 24."""
    import ctypes
    from hipzap import _native as N
    g = torch.Generator().manual_seed(K)
    M, Nn = 300, 384
    w = torch.randn(Nn, K, generator=g) * 0.05
    b = torch.randn(Nn, generator=g)
    x = torch.randn(M, K, generator=g)
    pw = F8.quantize_linear(C.pack_linear(w, b))
    pwd = F8.PackedFp8(pw.w8.to(DEV), pw.sw.to(DEV), pw.bias.to(DEV), pw.cin, pw.cout, pw.w8mx.to(DEV))
    x8, sx = F8.quant_rows(x.to(torch.bfloat16).to(DEV))
    outs = []
    for c in (24, cfg):
        out = torch.full((M, Nn), 7.0, device=DEV, dtype=torch.bfloat16)
        prm = F8.gemm_params(x8.data_ptr(), N.ptr(sx), pwd, M, out.data_ptr(), 0, "none", False, c, 1)
        N.check(N.lib().hz_launch_kernel(F8.K_GEMM_FP8, ctypes.byref(prm), N.stream_ptr()), f"gemm cfg {c}")
        torch.cuda.synchronize()
        outs.append(out.cpu())
    assert torch.equal(outs[0], outs[1]), f"cfg {cfg} differs from cfg 24 at K {K}"
