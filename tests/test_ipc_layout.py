"""CPU checks of the ipc transports' host logic (the kernels themselves run in
tests/test_ipc_gpu.py / test_ipc_p2p_gpu.py):

* the flag layouts of the one-sided lane and of the mailbox p2p: every flag
  has its own 64-B line inside the allocated area -- a flag outside it would
  be a stray store into a peer's memory;
* the planning of an IpcP2P group: queues per (direction, peer, channel) in
  issue order, sequence numbers advancing by mailbox pieces, zero-byte ops
  and aborted peers dropped, oversized groups refused."""
import pytest

from akka_allreduce_amd._native_loader import load

_n = load()


@pytest.mark.parametrize("N,np_,nslots,wpp", [(2, 1, 2, 1), (3, 7, 4, 8), (8, 64, 4, 8), (16, 128, 8, 16)])
def test_flag_layouts_disjoint_and_in_bounds(N, np_, nslots, wpp):
    d = _n.ipc_layout(N, np_, nslots, wpp)
    stride = d["stride"]
    for key, nbytes in (("lane_flags", d["lane_flag_bytes"]), ("p2p_flags", d["p2p_flag_bytes"])):
        idx = d[key]
        assert len(set(idx)) == len(idx), key  # one line per flag
        assert all(i % stride == 0 and 0 <= i for i in idx), key
        assert max(idx) * 4 + 4 <= nbytes, key  # inside the allocation
    assert d["window_slots"] == 2 * N + 1


def _plan(ops, n=4, piece=100, dead=(), send_seq=None, recv_seq=None):
    z = [0] * (n * 2)
    return _n.ipc_p2p_plan(ops, n, piece, [1 if p in dead else 0 for p in range(n)],
                           list(send_seq or z), list(recv_seq or z))


def test_plan_queues_keep_issue_order_and_count_pieces():
    # (send, peer, bytes, channel)
    ops = [(True, 1, 250, 0), (False, 1, 100, 0), (True, 2, 10, 0), (True, 1, 100, 0), (True, 1, 50, 1),
           (False, 1, 1, 0)]
    queues, send_seq, recv_seq, sent = _plan(ops)
    assert [[(s, p, c, b) for s, p, c, b, _ in q] for q in queues] == [
        [(True, 1, 0, 250), (True, 1, 0, 100)],  # send to 1 on channel 0, issue order kept
        [(False, 1, 0, 100), (False, 1, 0, 1)],
        [(True, 2, 0, 10)],
        [(True, 1, 1, 50)],
    ]
    # sequence numbers advance by ceil(bytes / piece) per op
    assert [seq for *_, seq in queues[0]] == [0, 3]
    assert [seq for *_, seq in queues[1]] == [0, 1]
    assert send_seq[1 * 2 + 0] == 4 and send_seq[1 * 2 + 1] == 1 and send_seq[2 * 2 + 0] == 1
    assert recv_seq[1 * 2 + 0] == 2
    assert sent == 250 + 10 + 100 + 50


def test_plan_continues_sequences_across_groups():
    q1, s1, r1, _ = _plan([(True, 3, 500, 1)])
    q2, s2, r2, _ = _plan([(True, 3, 1, 1), (False, 3, 1, 1)], send_seq=s1, recv_seq=r1)
    assert q1[0][0][4] == 0 and q2[0][0][4] == 5 and s2[3 * 2 + 1] == 6
    assert q2[1][0][4] == 0 and r2[3 * 2 + 1] == 1


def test_plan_drops_empty_ops_and_aborted_peers():
    queues, send_seq, recv_seq, sent = _plan([(True, 1, 0, 0), (True, 2, 64, 0), (False, 2, 64, 0),
                                              (True, 3, 64, 0)], dead=(2,))
    assert [[(s, p) for s, p, *_ in q] for q in queues] == [[(True, 3)]]
    assert sum(send_seq) == 1 and sum(recv_seq) == 0 and sent == 64


def test_plan_refuses_oversized_groups_and_bad_peers():
    with pytest.raises(Exception, match="ops in one group"):
        _plan([(True, 1, 8, 0)] * 81)
    with pytest.raises(Exception, match="peer out of range"):
        _plan([(True, 9, 8, 0)])
