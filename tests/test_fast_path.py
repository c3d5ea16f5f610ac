"""The collective-style fast path (ThresholdAllreduce.__call__ ->
AllreduceWorker._fast_allreduce -> native fast_round) at N=1 on the CPU:
whole-round bulk pass, counts table reused with a caller-owned output,
fresh buffers without one, and the engine's bookkeeping of every round
(rounds_completed, bulk rounds) -- the host path whose cost
profiles/r06/small_rounds/ measures."""
import torch

from akka_allreduce_amd.parallel import ThresholdAllreduce


def test_n1_rounds_with_reused_output_and_counts():
    S, C = 1000, 96  # kmax = 11 chunks, the last one short
    ar = ThresholdAllreduce(S, max_chunk_size=C, device="cpu", rank=0, world_size=1)
    buf = torch.empty(S)
    seen = []
    for r in range(4):
        x = torch.randn(S)
        o = ar(x, out=buf)
        assert o.data.data_ptr() == buf.data_ptr() and o.iteration == r
        assert torch.equal(o.data, x)
        assert o.counts_per_chunk.shape == (1, 11)
        assert bool((o.count == 1).all()) and o.count.numel() == S
        assert torch.equal(o.mean(), x)
        seen.append(o.counts_per_chunk.data_ptr())
    assert len(set(seen)) == 1  # one counts table travels with the one output buffer
    st = ar.worker.state()
    assert st["stats"]["rounds_completed"] == 4 and st["stats"]["bulk_rounds"] == 4
    assert st["round"] == 4 and ar.worker.fast_rounds == 4


def test_n1_rounds_without_output_get_fresh_buffers():
    S = 300
    ar = ThresholdAllreduce(S, max_chunk_size=64, device="cpu", rank=0, world_size=1)
    xs = [torch.randn(S) for _ in range(3)]
    outs = [ar(x) for x in xs]
    assert len({o.data.data_ptr() for o in outs}) == 3
    assert len({o.counts_per_chunk.data_ptr() for o in outs}) == 3
    for x, o in zip(xs, outs):
        assert torch.equal(o.data, x) and bool((o.count == 1).all())


def test_n1_bad_output_buffer_is_rejected():
    ar = ThresholdAllreduce(128, max_chunk_size=32, device="cpu", rank=0, world_size=1)
    x = torch.randn(128)
    for bad in (torch.empty(127), torch.empty(128, dtype=torch.float64), torch.empty(256)[::2]):
        try:
            ar(x, out=bad)
        except ValueError:
            continue
        raise AssertionError("a bad output buffer was accepted")
    assert torch.equal(ar(x, out=torch.empty(128)).data, x)  # and the worker still runs rounds


def test_n1_bf16_in_place():
    S = 512
    ar = ThresholdAllreduce(S, max_chunk_size=100, dtype=torch.bfloat16, device="cpu", rank=0, world_size=1)
    x = torch.randn(S).to(torch.bfloat16)
    want = x.clone()
    o = ar(x, out=x)  # in place: input and output are one buffer
    assert torch.equal(o.data, want)
