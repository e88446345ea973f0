"""Dynamic request batching (serve/batcher.py) on the CPU: coalescing, ordering, errors."""
import threading

import pytest
import torch

from hipzap.serve.batcher import DynamicBatcher


def _concurrent(fn, inputs):
    out = [None] * len(inputs)
    start = threading.Barrier(len(inputs))

    def run(i):
        start.wait()
        out[i] = fn(inputs[i])
    th = [threading.Thread(target=run, args=(i,)) for i in range(len(inputs))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=30)
    return out


def test_coalesces_concurrent_requests_and_slices_results():
    sizes = []

    def run(x):
        sizes.append(x.shape[0])
        return x * 2 + 1

    b = DynamicBatcher(run, max_batch=8, max_wait_ms=200)
    xs = [torch.full((1, 3), float(i)) for i in range(8)]
    ys = _concurrent(b, xs)
    b.close()
    for x, y in zip(xs, ys):
        assert torch.equal(y, x * 2 + 1)  # every caller gets its own rows back
    assert sum(sizes) == 8 and max(sizes) > 1  # at least one multi-request batch
    assert b.requests == 8 and b.batches == len(sizes)


def test_full_batch_dispatches_without_waiting():
    import time
    b = DynamicBatcher(lambda x: x, max_batch=2, max_wait_ms=10_000)
    t0 = time.perf_counter()
    ys = _concurrent(b, [torch.ones(1, 1), torch.zeros(1, 1)])
    assert time.perf_counter() - t0 < 5 and sorted(float(y) for y in ys) == [0.0, 1.0]
    b.close()


def test_lone_request_waits_at_most_max_wait():
    import time
    b = DynamicBatcher(lambda x: x + 1, max_batch=16, max_wait_ms=20)
    t0 = time.perf_counter()
    y = b(torch.zeros(2, 1))
    assert torch.equal(y, torch.ones(2, 1)) and time.perf_counter() - t0 < 2
    b.close()


def test_batches_never_exceed_max_batch():
    sizes = []

    def run(x):
        sizes.append(x.shape[0])
        return x

    b = DynamicBatcher(run, max_batch=4, max_wait_ms=100)
    ys = _concurrent(b, [torch.full((3, 1), float(i)) for i in range(5)])  # 3+3 > 4: never merged
    b.close()
    assert all(s <= 4 for s in sizes) and [float(y[0]) for y in ys] == [0.0, 1.0, 2.0, 3.0, 4.0]
    with pytest.raises(ValueError):
        DynamicBatcher(run, max_batch=4).submit(torch.zeros(5, 1))


def test_error_reaches_every_request_of_the_batch():
    def run(x):
        raise RuntimeError("device fault")

    b = DynamicBatcher(run, max_batch=4, max_wait_ms=100)
    errs = _concurrent(lambda x: _catch(b, x), [torch.zeros(1, 1)] * 3)
    b.close()
    assert all(isinstance(e, RuntimeError) and "device fault" in str(e) for e in errs)


def _catch(b, x):
    try:
        return b(x)
    except Exception as e:  # noqa: BLE001
        return e


def test_vision_backend_batching_config_cpu_path_unaffected():
    """On the CPU backend the batching block is ignored (no engine): plain eager forward."""
    from hipzap.serve.server import VisionBackend
    from hipzap.serve.settings import ModelSpec
    from hipzap.models import registry
    torch.manual_seed(0)
    sd = registry.get("resnet18").make_model().state_dict()
    be = VisionBackend("resnet18", sd, "cpu", "cpu", ModelSpec("resnet18", batch=4,
                                                               extra={"batching": {"max_wait_ms": 1}}), False)
    assert be.batcher is None
    assert be(torch.randn(1, 3, 32, 32)).shape == (1, 1000)
