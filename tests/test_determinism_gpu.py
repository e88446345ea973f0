"""Deterministic served logits. The default ResNet-50 program's layer3 /
layer4 seams and K-split 3x3 convs sum partial products across workgroups with memory-side float
atomics; every term they add is first rounded to a multiple of 2^-10 (csrc/common.h hz_fixq), so
the sums are exact and independent of arrival order. 1,008 replays of one image spread over 16
concurrent request contexts (the bench's serving shape, through the native request executor) and
a second, independently built engine all return the same bits."""
import threading

import pytest
import torch

from hipzap.engine import fusion
from hipzap.engine.engine import Engine
from hipzap.models import registry
from hipzap.models.resnet import randomize_bn

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def packed():
    torch.manual_seed(0)
    a = registry.get("resnet50")
    sd = randomize_bn(a.make_model()).eval().state_dict()
    params, kw = a.pack({k: v.to(DEV) for k, v in sd.items()}, torch.device(DEV))
    return params, dict(kw, input_uint8=True)


def test_default_program_has_the_atomic_launches(packed):
    params, kw = packed
    eng = Engine("resnet50", params, DEV, batch=1, num_contexts=1, arch_kw=kw)
    kinds = [f.kind for f in eng.contexts[0].fused.values()]
    assert kinds.count("seam") == 8 and kinds.count("kconv") == 9, kinds  # (fusion.DEFAULT)
    assert fusion.enabled_kinds() >= {"seam", "kconv"}


def test_replays_under_16_streams_are_bitwise_identical(packed):
    params, kw = packed
    eng = Engine("resnet50", params, DEV, batch=1, num_contexts=16, arch_kw=kw, host_io=True, zero_copy="all")
    eng.ensure_contexts()
    x = torch.randint(0, 256, (1, 224, 224, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(7))
    y0 = eng.infer(x).clone()
    assert torch.isfinite(y0).all()
    outs, errs = [], []
    lock = threading.Lock()

    def client(k):
        try:
            mine = [eng.infer(x).clone() for _ in range(63)]
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))
            return
        with lock:
            outs.extend(mine)

    th = [threading.Thread(target=client, args=(k,)) for k in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errs, errs[:3]
    assert len(outs) == 16 * 63
    bad = sum(not torch.equal(o, y0) for o in outs)
    assert bad == 0, f"{bad} of {len(outs)} replays differ from the first (max diff " \
                     f"{max((o - y0).abs().max().item() for o in outs)})"
    # an independently built engine (own arena, own graph) gives the same bits
    other = Engine("resnet50", params, DEV, batch=1, num_contexts=1, arch_kw=kw, host_io=True, zero_copy="all")
    assert torch.equal(other.infer(x), y0)
