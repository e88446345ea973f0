"""FP8 (OCP e4m3fn) quantisation + fp8 MFMA GEMM on MI355X."""
import pytest
import torch

from hipzap.engine.engine import Engine
from hipzap.models import vit
from hipzap.ops import conv as C
from hipzap.ops import fp8 as F8

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


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
    torch.manual_seed(0)
    m = vit.make_model(num_labels=1000)
    eng = Engine.from_state_dict("vit-b16-fp8", m.state_dict(), DEV, batch=4)
    x = torch.randn(4, 3, 224, 224)
    out = eng.infer(x)
    with torch.no_grad():
        ref = m(pixel_values=x).logits
    rel = ((out - ref).abs().max() / ref.abs().max()).item()
    assert rel < 0.25, rel
    cos = torch.nn.functional.cosine_similarity(out, ref, dim=1)
    assert cos.min() > 0.97, cos


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
