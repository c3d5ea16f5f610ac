"""Rank program for tests/test_racecheck.py (torch.distributed.run, gloo, CPU):
ThresholdAllreduce rounds through the native fast path (caller buffers bound
in C++) with the stream race checker on (AKKA_RACECHECK=1) and a modelled
caller stream.  The caller writes the input, hands over output / counts
memory that earlier work on its stream may still write, and reads the results
on its stream.  Writes <out_dir>/rank<i>.json."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    S, C, lane, rounds, out_dir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), sys.argv[5]
    offstream = len(sys.argv) > 6 and sys.argv[6] == "offstream"
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    from akka_allreduce_amd.parallel import ThresholdAllreduce

    ar = ThresholdAllreduce(S, max_chunk_size=C, device=torch.device("cpu"), lane=lane)
    w = ar.worker
    assert w._core.models_streams(), "race checking is not on"
    hs = w.host_stream = w._core.create_stream()
    orig = w._alloc_counts

    def counts_from_recycled_memory():
        c = orig()
        w._core.declare_access(hs, c.data_ptr(), c.numel() * 4, True, "caller.pending_write")
        return c

    w._alloc_counts = counts_from_recycled_memory
    out = torch.empty(S)
    exact = []
    for r in range(rounds):
        x = torch.full((S,), float(rank + 1 + r))
        w._core.declare_access(hs, x.data_ptr(), S * 4, True, "caller.input_write")
        w._core.declare_access(hs, out.data_ptr(), S * 4, True, "caller.pending_write")
        o = ar(x, out=out)
        # offstream: the caller reads the result on another stream, without a wait (a bug to flag)
        rs = w._core.create_stream() if offstream else hs
        w._core.declare_access(rs, o.data.data_ptr(), S * 4, False, "caller.read")
        pc = o.counts_per_chunk
        w._core.declare_access(hs, pc.data_ptr(), pc.numel() * 4, False, "caller.read")
        want = float(sum(k + 1 + r for k in range(world)))
        exact.append(bool((o.data == want).all()) and bool((pc == world).all()))
    st = ar.state()["link"]
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump({"rank": rank, "exact": exact, "races": w._core.race_count(),
                   "reports": w._core.race_reports()[:6], "fast_rounds": w.fast_rounds,
                   "collective_rounds": st.get("collective_rounds"),
                   "exact_step_rounds": st.get("exact_step_rounds")}, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
