"""Request-context streams (engine.py ``stream_kind``): an engine of 2-4 contexts gets fresh
high-priority streams (HIP's separate set of queues for that priority), more contexts share
torch's stream pool.
The logits do not depend on which: every context of a dedicated-queue engine gives bitwise the
pooled engine's output, and concurrent replays on the dedicated queues stay correct."""
import pytest
import torch

from hipzap.engine.engine import Engine, stream_kind
from hipzap.models import registry
from hipzap.models.resnet import randomize_bn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def test_stream_kind_policy(monkeypatch):
    monkeypatch.delenv("HIPZAP_STREAM_KIND", raising=False)
    assert [stream_kind(n) for n in (1, 2, 4, 5, 16)] == ["torch", "hiprio", "hiprio", "torch", "torch"]
    assert stream_kind(4, "torch") == "torch"  # an engine's own choice wins over the default
    monkeypatch.setenv("HIPZAP_STREAM_KIND", "native")
    assert stream_kind(4) == "native"
    monkeypatch.setenv("HIPZAP_STREAM_KIND", "bogus")
    with pytest.raises(ValueError):
        stream_kind(2)


def test_dedicated_queue_contexts_match_pooled_bitwise(monkeypatch):
    torch.manual_seed(0)
    sd = randomize_bn(registry.get("resnet18").make_model()).eval().state_dict()
    x = torch.randn(2, 3, 224, 224, generator=torch.Generator().manual_seed(5))
    monkeypatch.setenv("HIPZAP_STREAM_KIND", "torch")
    ref_eng = Engine.from_state_dict("resnet18", sd, DEV, batch=2, num_contexts=1)
    ref = ref_eng.infer(x)
    monkeypatch.delenv("HIPZAP_STREAM_KIND")
    # a device-I/O engine keeps torch's pooled streams by default (its callers' stream waits)
    eng_d = Engine.from_state_dict("resnet18", sd, DEV, batch=2, num_contexts=3, host_io=False)
    assert not any(isinstance(s, torch.cuda.ExternalStream) for s in eng_d.streams)
    del eng_d
    eng = Engine.from_state_dict("resnet18", sd, DEV, batch=2, num_contexts=3, host_io=False, stream_kind="hiprio")
    # high-priority streams of its own (HIP's separate queue set for that priority)
    assert all(isinstance(s, torch.cuda.ExternalStream) for s in eng.streams)
    assert len({s.cuda_stream for s in eng.streams}) == 3
    xd = x.to(DEV)
    outs = [eng.infer_device(xd, i).clone() for i in range(3)]
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o.cpu().reshape(ref.shape), ref)
    eng.bench(20)  # every context replayed concurrently on its own queue
    outs2 = [c.output.clone() for c in eng.contexts]
    torch.cuda.synchronize()
    for o in outs2:
        assert torch.equal(o.cpu().reshape(ref.shape), ref)
    xd2 = x.to(DEV)
    eng.infer_device(xd2, 1)  # a tensor recorded on a pooled stream, freed after the engine
    del eng
    import gc
    gc.collect()
    del xd2
    torch.cuda.synchronize()
