"""RCCL data-plane checks that run on ONE MI355X (1-rank communicators).

RCCL refuses two ranks on one card, so the N>1 p2p schedule is validated on
the CPU simulator and the loopback transports; what one GPU CAN show about
the real library is covered here:

* the communicator reports (ncclCommCount / ncclCommUserRank /
  ncclCommCuDevice) what the transport was built with -- the same values
  bench.py prints as ``rccl_nranks`` / ``rank_devices`` at N>1;
* several sends and receives to the SAME peer inside one group are matched in
  issue order (the StreamLink's last step carries scatter, broadcast and
  counts to each peer in one group: stream_link.cpp);
* the async-error check is clean after real traffic.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ep(native):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    return native.rccl_endpoint(native.rccl_unique_id(), 0, 1, 0)


def test_rccl_comm_reports_what_it_was_built_with(native, ep):
    info = ep.info()
    assert info == {"kind": "rccl", "nranks": 1, "rank": 0, "device": 0, "comms": 1}
    assert native.rccl_version().count(".") == 2
    ep.check()


def test_rccl_same_peer_ops_match_in_issue_order(ep):
    dev = torch.device("cuda", 0)
    # three sends + three receives to one peer in one group, sizes all different:
    # any out-of-order match would mis-size or mis-route a buffer
    sizes = [3 << 20, 4096, (1 << 20) + 64]
    src = [torch.arange(n // 4, device=dev, dtype=torch.float32) + 1000 * i for i, n in enumerate(sizes)]
    dst = [torch.full((n // 4,), -1.0, device=dev) for n in sizes]
    ops = []
    for a, b, n in zip(src, dst, sizes):
        ops.append((True, 0, a.data_ptr(), n))
    for a, b, n in zip(src, dst, sizes):
        ops.append((False, 0, b.data_ptr(), n))
    s = torch.cuda.current_stream(dev)
    ep.group(s.cuda_stream, ops)
    torch.cuda.synchronize()
    for a, b in zip(src, dst):
        assert torch.equal(a, b)
    ep.check()


def test_rccl_n8_step_shape_exact(ep):
    """The N=8 StreamLink step shape (7 peers x {scatter, bcast} sends and as
    many receives = 28 ops) in one group, 1 MiB each, is byte-exact."""
    dev = torch.device("cuda", 0)
    n = 1 << 20
    src = [torch.randn(n // 4, device=dev) for _ in range(14)]
    dst = [torch.empty_like(t) for t in src]
    ops = []
    for a, b in zip(src, dst):
        ops.append((True, 0, a.data_ptr(), n))
        ops.append((False, 0, b.data_ptr(), n))
    ep.group(torch.cuda.current_stream(dev).cuda_stream, ops)
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(src, dst))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_rccl_collective_lane_calls(ep, dtype):
    """The whole-round lane's two RCCL calls (reduce-scatter, then in-place
    all-gather) with the types the engine passes; on a 1-rank communicator
    both are copies, so the result must equal the input bit for bit."""
    dev = torch.device("cuda", 0)
    assert ep.has_collectives()
    n = (1 << 20) + 16
    x = torch.randn(n, device=dev).to(dtype)
    out = torch.empty_like(x)
    s = torch.cuda.current_stream(dev).cuda_stream
    name = "bfloat16" if dtype == torch.bfloat16 else "float32"
    ep.reduce_scatter(s, x.data_ptr(), out.data_ptr(), n, name)
    ep.all_gather(s, out.data_ptr(), out.data_ptr(), n, name)
    torch.cuda.synchronize()
    assert torch.equal(out, x)
    ep.check()


@pytest.mark.parametrize("graphs", [False, True])
def test_shape_rehearsal_exact_schedule_and_graph_replay(graphs):
    """The N=8 exact step schedule through real RCCL on one GPU
    (RcclShapeP2P: rank 0 of 8 posing, every op to itself).  With a constant
    input every slot and every broadcast carries that constant whatever the
    pairing, so the output must be 8*c with count 8 -- round after round,
    also when the rounds replay a captured HIP graph with new input values."""
    from akka_allreduce_amd import AllreduceWorker, InitWorkers
    from akka_allreduce_amd.parallel.collective import _RemoteRank

    dev = torch.device("cuda", 0)
    n, C = 8, 1024
    S = n * 4 * C + n * 8  # even split, short last chunk in every block
    w = AllreduceWorker(None, None, device=dev, transport="stream", transport_spec=("rccl_shape", 0, n),
                        strict=True, name="shape")
    w.tell(InitWorkers({i: (w if i == 0 else _RemoteRank(i)) for i in range(n)}, n, None, 0, 1.0, 1.0, 2, S, C))
    w.set_lane("p2p")
    w.set_graphs(graphs)
    x = torch.empty(S, device=dev)
    out = torch.empty(S, device=dev)
    for r in range(12):  # 3 ring rows: each key is captured at its 2nd round, replayed from its 3rd
        x.fill_(float(r + 1))
        o = w.allreduce(x, out=out)
        torch.cuda.synchronize()
        assert torch.equal(o.data, torch.full_like(x, 8.0 * (r + 1))), r
        assert bool((o.count == n).all())
    st = w.state()["link"]
    assert st["exact_step_rounds"] == 12 and "graph_error" not in st, st
    if graphs:
        assert st["graph_captures"] == 3 and st["graph_replays"] == 6, st
    w.close()
