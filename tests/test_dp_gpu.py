"""Data-parallel scatter/gather on the GPU (SURVEY.md §4.2 T-comm-gpu):
DPExecutor over real Engines, including the stream ordering between the caller's stream and the
engine's context stream (the round-1 race: the context stream did not wait for the scatter, the
caller did not wait for the replay)."""
import pytest
import torch

from hipzap.engine.engine import Engine
from hipzap.models import registry
from hipzap.models.resnet import randomize_bn
from hipzap.parallel.dp import DPExecutor
from hipzap.parallel.loopback import run_ranks

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def sd():
    torch.manual_seed(0)
    return randomize_bn(registry.get("resnet18").make_model()).eval().state_dict()


def _images(n, seed):
    return torch.randn(n, 3, 224, 224, generator=torch.Generator().manual_seed(seed))


def test_dp_world1_matches_engine_bitwise_under_a_caller_stream(sd):
    """32 images through DPExecutor (world 1) == the same batch-32 engine's host path, bitwise,
    for several back-to-back steps issued on a non-default caller stream."""
    eng = Engine.from_state_dict("resnet18", sd, DEV, batch=32, num_contexts=1, host_io=False)
    ex = DPExecutor(lambda xs: eng.infer_device(xs), 32, tuple(eng.contexts[0].input.shape[1:]),
                    tuple(eng.contexts[0].output.shape[1:]), DEV)
    ref_eng = Engine.from_state_dict("resnet18", sd, DEV, batch=32, num_contexts=1)
    caller = torch.cuda.Stream(DEV)
    outs, xs = [], [_images(32, s) for s in range(4)]
    with torch.cuda.stream(caller):
        for x in xs:  # no host sync between steps: ordering must come from the stream waits
            outs.append(ex.step(x.to(DEV, non_blocking=True)))
    caller.synchronize()
    for x, y in zip(xs, outs):
        ref = ref_eng.infer(x)
        assert torch.equal(y.cpu().reshape(ref.shape), ref)


def test_dp_uneven_batch_pads_and_slices(sd):
    eng = Engine.from_state_dict("resnet18", sd, DEV, batch=8, num_contexts=1, host_io=False)
    ex = DPExecutor(lambda xs: eng.infer_device(xs), 8, tuple(eng.contexts[0].input.shape[1:]),
                    tuple(eng.contexts[0].output.shape[1:]), DEV)
    x = _images(5, 7).to(DEV)
    y = ex.step(x)
    full = torch.cat([x, torch.zeros(3, *x.shape[1:], device=DEV)])
    ref = ex.step(full)
    assert y.shape[0] == 5 and torch.equal(y, ref[:5])


def test_dp_loopback_world4_with_gpu_replicas(sd):
    """4 ranks (loopback threads, one Engine replica each on the GPU): rank 0 scatters a global
    batch of 32, every rank runs its shard of 8, logits gathered back == each shard run alone."""
    world, shard = 4, 8
    engines = [Engine.from_state_dict("resnet18", sd, DEV, batch=shard, num_contexts=1, host_io=False)
               for _ in range(world)]
    xg = _images(world * shard, 11).to(DEV)
    ref = torch.cat([engines[0].infer_device(xg[r * shard:(r + 1) * shard]).clone() for r in range(world)])
    torch.cuda.synchronize()

    def rank_fn(comm):
        torch.cuda.set_device(DEV)
        eng = engines[comm.rank]
        ex = DPExecutor(lambda xs: eng.infer_device(xs), shard, tuple(eng.contexts[0].input.shape[1:]),
                        tuple(eng.contexts[0].output.shape[1:]), DEV, comm=comm)
        out = ex.step(xg if comm.rank == 0 else None)
        torch.cuda.synchronize()
        return out

    res = run_ranks(world, rank_fn, timeout_s=120)
    for r in res:
        assert not isinstance(r, BaseException), r
    assert torch.equal(res[0].reshape(ref.shape), ref)
    assert all(r is None for r in res[1:])


def test_dp_pipeline_three_in_flight_matches_engine_bitwise(sd):
    """DPPipeline over three captured contexts (three batch-8 steps in flight on their own streams,
    issued from a non-default caller stream with no host sync): every step's logits equal the
    host path's for its own images, bitwise and in order (the slot reuse and the stream waits)."""
    from hipzap.parallel.dp import DPPipeline
    eng = Engine.from_state_dict("resnet18", sd, DEV, batch=8, num_contexts=3, host_io=False)
    pipe = DPPipeline(eng.pipeline_slots(), 8, tuple(eng.contexts[0].output.shape[1:]), DEV)
    ref_eng = Engine.from_state_dict("resnet18", sd, DEV, batch=8, num_contexts=1)
    xs = [_images(8 - (i % 3 == 2), 100 + i) for i in range(7)]
    caller = torch.cuda.Stream(DEV)
    outs = []
    with torch.cuda.stream(caller):
        for x in xs:
            y = pipe.submit(x.to(DEV, non_blocking=True))
            if y is not None:
                outs.append(y.clone())
        outs += [y.clone() for y in pipe.flush()]
    caller.synchronize()
    assert len(outs) == len(xs)
    for x, y in zip(xs, outs):
        full = torch.cat([x, torch.zeros(8 - x.shape[0], *x.shape[1:])]) if x.shape[0] < 8 else x
        ref = ref_eng.infer(full)[:x.shape[0]]
        assert torch.equal(y.cpu().reshape(ref.shape), ref)
