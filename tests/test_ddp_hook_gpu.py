"""The DDP hook on the GPU is asynchronous: it queues the round, the
count-weighted mean and the future's ready event in stream order and returns
without waiting for the GPU -- so DDP overlaps bucket communication with the
rest of the backward pass, like its own allreduce hook."""
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Bucket:
    """The part of dist.GradBucket the hook reads."""

    def __init__(self, t):
        self._t = t

    def buffer(self):
        return self._t


@pytest.mark.parametrize("async_op", [True, False])
def test_hook_returns_before_the_gpu_ran_the_round(async_op):
    from akka_allreduce_amd.parallel.ddp import ThresholdHookState, threshold_allreduce_hook

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g = torch.randn(1 << 20, device=dev)
    state = ThresholdHookState(max_chunk_size=1 << 16, async_op=async_op)
    # warm up: engine creation, first round
    threshold_allreduce_hook(state, _Bucket(g.clone())).wait()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream(dev)
    torch.cuda._sleep(200_000_000)  # keep the stream busy for a while (~0.1 s)
    fut = threshold_allreduce_hook(state, _Bucket(g))
    pending = not s.query()
    got = fut.wait()
    torch.cuda.synchronize()
    assert pending  # the hook never synchronized the stream
    assert torch.equal(got, g)  # N=1: the mean over the one contributor is the gradient itself
    assert state.async_rounds == (2 if async_op else 0)
