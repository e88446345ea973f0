"""Dynamic-batching request executor (csrc/executor.cpp hz_exec_create_batched): bs=1 requests
from concurrent threads share batched replays; every request gets ITS OWN row back (MI355X)."""
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_dynamic_batching_rows_match_single_requests():
    from hipzap.engine.engine import Engine
    from hipzap.models import registry
    from hipzap.models.resnet import randomize_bn
    torch.manual_seed(0)
    adapter = registry.get("resnet50")
    sd = randomize_bn(adapter.make_model()).eval().state_dict()
    params, arch_kw = adapter.pack({k: v.to(DEV) for k, v in sd.items()}, DEV)
    arch_kw = dict(arch_kw, input_uint8=True)
    one = Engine("resnet50", params, DEV, batch=1, num_contexts=1, arch_kw=arch_kw, zero_copy="all")
    bat = Engine("resnet50", params, DEV, batch=4, num_contexts=2, arch_kw=arch_kw, zero_copy="all")
    ex = bat.batched_executor(max_wait_us=500.0)
    shape = tuple(one.contexts[0].host_input.shape)
    g = torch.Generator().manual_seed(1)
    imgs = [torch.randint(0, 256, shape, generator=g, dtype=torch.uint8) for _ in range(24)]
    refs = [one.infer(x).float().reshape(-1) for x in imgs]
    ho = one.contexts[0].host_output
    outs = [torch.zeros(ho.numel(), dtype=ho.dtype) for _ in imgs]
    assert ex.out_bytes == ho.numel() * ho.element_size()
    errs = []

    def client(c):
        try:
            for rep in range(3):
                for i in range(c, len(imgs), 8):
                    ex.submit([imgs[i].data_ptr()], outs[i].data_ptr())
                    o = outs[i].float()
                    err = (o - refs[i]).abs().max().item() / refs[i].abs().max().item()
                    if err > 3e-2 or o.argmax() != refs[i].argmax():
                        errs.append((c, i, rep, err))
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=client, args=(c,)) for c in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in th), "executor hung"
    assert not errs, errs[:5]
    st = ex.stats()
    assert st["served"] >= 72 and st["batches"] < st["served"], st  # some replays carried several requests
    ex.close()


def test_multi_row_requests_share_batches_with_single_rows():
    """hz_exec_submit_rows: one thread submits m consecutive rows (m = 1..4 on a batch-4 plan, so
    chunks straddle partly filled batches) while other threads submit single rows; every row of
    every request comes back as its own image's logits."""
    from hipzap.engine.engine import Engine
    from hipzap.models import registry
    from hipzap.models.resnet import randomize_bn
    torch.manual_seed(0)
    adapter = registry.get("resnet50")
    sd = randomize_bn(adapter.make_model()).eval().state_dict()
    params, arch_kw = adapter.pack({k: v.to(DEV) for k, v in sd.items()}, DEV)
    arch_kw = dict(arch_kw, input_uint8=True)
    one = Engine("resnet50", params, DEV, batch=1, num_contexts=1, arch_kw=arch_kw, zero_copy="all")
    bat = Engine("resnet50", params, DEV, batch=4, num_contexts=2, arch_kw=arch_kw, zero_copy="all")
    ex = bat.batched_executor(max_wait_us=300.0)
    shape = tuple(one.contexts[0].host_input.shape)[1:]
    g = torch.Generator().manual_seed(2)
    imgs = torch.randint(0, 256, (16,) + shape, generator=g, dtype=torch.uint8)
    refs = torch.stack([one.infer(imgs[i: i + 1]).float().reshape(-1) for i in range(16)])
    ho = one.contexts[0].host_output
    with pytest.raises(ValueError):
        ex.submit_rows([imgs.data_ptr()], 5, 0)
    errs = []

    def check(i0, m, out):
        for r in range(m):
            o, ref = out[r].float(), refs[i0 + r]
            err = (o - ref).abs().max().item() / ref.abs().max().item()
            if err > 3e-2 or o.argmax() != ref.argmax():
                errs.append((i0, m, r, err))

    def multi(c):
        try:
            for rep in range(4):
                m = 1 + (c + rep) % 4
                i0 = (3 * c + rep) % (16 - m + 1)
                x = imgs[i0: i0 + m].contiguous()
                out = torch.zeros((m, ho.numel()), dtype=ho.dtype)
                ex.submit_rows([x.data_ptr()], m, out.data_ptr())
                check(i0, m, out)
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    def single(c):
        try:
            for i in range(c, 16, 3):
                out = torch.zeros((1, ho.numel()), dtype=ho.dtype)
                ex.submit([imgs[i].data_ptr()], out.data_ptr())
                check(i, 1, out)
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=multi, args=(c,)) for c in range(4)] + \
         [threading.Thread(target=single, args=(c,)) for c in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in th), "executor hung"
    assert not errs, errs[:5]
    st = ex.stats()
    assert st["served"] == sum(1 + (c + rep) % 4 for c in range(4) for rep in range(4)) + 16, st
    ex.close()
