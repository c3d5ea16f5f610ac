"""Membership epochs of the device data plane (the reference
removes a dead worker, M:46-52, and re-InitWorkers replaces the peer map,
W:87-89).  On an RCCL data plane a worker cannot leave a communicator it
shares with a dead rank, so the master starts a new epoch: the survivors get
a re-InitWorkers carrying a NEW unique id and the survivor list, and build a
communicator over themselves (engine ids map to communicator ranks by their
index in the list)."""
import pytest
import torch

from akka_allreduce_amd import AllreduceMaster
from akka_allreduce_amd.messages import InitWorkers, StartAllreduce, WorkerTerminated
from akka_allreduce_amd.testing import TestProbe


def _uid_for(master):
    def info():
        members = sorted(master.workers)
        return {"kind": "rccl", "uid": bytes([len(members)] + members) * 8}
    return info


def test_master_starts_new_epoch_after_death():
    m = AllreduceMaster(4, 0.75, 0.75, 0.75, 1, 64, 10, 8)
    m.transport_info = _uid_for(m)
    probes = [TestProbe(f"w{i}") for i in range(4)]
    for p in probes:
        m.member_up(p)
    first = {}
    for i, p in enumerate(probes):
        init = p.receive_one()
        assert isinstance(init, InitWorkers) and init.transport["members"] == [0, 1, 2, 3]
        first[i] = init.transport["uid"]
        p.expect_msg(StartAllreduce(0))
    m.terminated(3)
    for i in range(3):
        p = probes[i]
        p.expect_msg(WorkerTerminated(3))
        init = p.receive_one()
        assert isinstance(init, InitWorkers)
        assert sorted(init.workers) == [0, 1, 2] and init.transport["members"] == [0, 1, 2]
        assert init.transport["uid"] != first[i]  # a new communicator, not the old one
    assert not probes[3].queue


def test_cpu_data_plane_gets_no_epoch():
    """Without a device transport the peer map alone changes (reference behaviour)."""
    m = AllreduceMaster(3, 1.0, 1.0, 1.0, 1, 30, 5, 5)
    probes = [TestProbe(f"w{i}") for i in range(3)]
    for p in probes:
        m.member_up(p)
    for p in probes:
        p.receive_one()
        p.receive_one()
    m.terminated(2)
    for p in probes[:2]:
        p.expect_msg(WorkerTerminated(2))
        assert not p.queue


@pytest.mark.gpu
def test_rccl_epoch_rebuild_on_one_gpu(native):
    """One GPU: worker 0 of a 2-worker geometry whose communicator holds only
    itself (members [0]); a re-InitWorkers with a new unique id rebuilds it
    (abort + ncclCommInitRank over the members) and rounds keep completing
    from the member's own contribution (thresholds 0.5)."""
    from akka_allreduce_amd import AllreduceWorker

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    S, C = 1 << 12, 256
    w = AllreduceWorker(None, None, device=dev, transport="stream", strict=True, name="epoch0")
    init = InitWorkers({0: w}, 2, None, 0, 0.5, 0.5, 1, S, C)
    init.transport = {"kind": "rccl", "uid": native.rccl_unique_id(), "members": [0]}
    w.tell(init)
    assert w._core.p2p_info()["nranks"] == 1

    def one_round():
        x = torch.full((S,), 3.0, device=dev)
        o = w.allreduce(x)
        torch.cuda.synchronize()
        half = (S + 1) // 2
        assert torch.equal(o.data[:half], x[:half]) and bool((o.count[:half] == 1).all())
        assert bool((o.count[half:] == 0).all())

    one_round()
    again = InitWorkers({0: w}, 2, None, 0, 0.5, 0.5, 1, S, C)
    again.transport = {"kind": "rccl", "uid": native.rccl_unique_id(), "members": [0]}
    w.tell(again)
    assert w.epochs == 1 and w._core.p2p_info() == {"kind": "rccl", "nranks": 1, "rank": 0, "device": 0,
                                                     "comms": 1}
    one_round()
    w.close()
