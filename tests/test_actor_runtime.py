"""The TCP actor runtime (akka_allreduce_amd/parallel/actors.py): one
selector-driven dispatcher per node, frames split out of each ``recv``, and
batched sends.  What the reference gets from Akka remoting and these tests
pin: per sender->receiver FIFO order (SPEC:590, SPEC:721), one message at a
time in ``receive``, local messages from other threads, a clean stop."""
import threading
import time

import torch

from akka_allreduce_amd.messages import ScatterBlock, StartAllreduce
from akka_allreduce_amd.parallel import wire
from akka_allreduce_amd.parallel.actors import Node


class Recorder:
    def __init__(self, want):
        self.got = []
        self.want = want
        self.done = threading.Event()
        self.inside = 0
        self.overlap = False

    def receive(self, msg):
        self.inside += 1
        self.overlap |= self.inside > 1
        self.got.append(msg)
        time.sleep(0)  # let another thread in, if any could deliver concurrently
        self.inside -= 1
        if len(self.got) >= self.want:
            self.done.set()


def test_batches_and_singles_keep_per_pair_fifo_order():
    """Two senders, each mixing single sends and batches, to one receiver:
    each sender's messages arrive in its own order, never two at once."""
    n_per = 600
    rec = Recorder(2 * n_per)
    dst = Node(name="dst").start(rec)
    srcs = [Node(name=f"src{i}").start(Recorder(0)) for i in range(2)]

    def send_all(i, node):
        k = 0
        while k < n_per:
            if k % 3 == 0:  # a batch of up to 5 (one write on the wire)
                m = min(5, n_per - k)
                node.send_many(dst.address, [StartAllreduce(i * 100000 + k + j) for j in range(m)])
                k += m
            else:
                node.send(dst.address, StartAllreduce(i * 100000 + k))
                k += 1

    ts = [threading.Thread(target=send_all, args=(i, n)) for i, n in enumerate(srcs)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert rec.done.wait(30), len(rec.got)
    for i in range(2):
        mine = [m.round - i * 100000 for m in rec.got if m.round // 100000 == i]
        assert mine == list(range(n_per)), mine[:20]
    assert not rec.overlap
    for n in srcs + [dst]:
        n.stop()
        n.join(5)


def test_frames_split_across_and_within_recvs():
    """FrameReader.feed: a frame cut anywhere, several frames in one chunk."""
    frames = [wire.encode(StartAllreduce(r), lambda ref: None) for r in range(5)]
    frames.append(wire.encode(ScatterBlock(torch.arange(7, dtype=torch.float32), 0, 1, 2, 3), lambda ref: None))
    blob = b"".join(frames)
    for cut in (1, 3, 4, 5, 17, len(blob) - 1):
        r = wire.FrameReader()
        bodies = r.feed(blob[:cut]) + r.feed(blob[cut:])
        msgs = [wire.decode(b, lambda a: None) for b in bodies]
        assert [m.round for m in msgs] == [0, 1, 2, 3, 4, 3]
        assert torch.equal(msgs[-1].value, torch.arange(7, dtype=torch.float32))


def test_local_posts_from_other_threads_and_stop():
    """mailbox.put from another thread wakes a dispatcher blocked on its
    sockets; stop() ends it and a later post is a no-op."""
    rec = Recorder(3)
    node = Node(name="solo").start(rec)
    for r in range(3):
        threading.Thread(target=node.mailbox.put, args=(StartAllreduce(r),)).start()
    assert rec.done.wait(10)
    assert sorted(m.round for m in rec.got) == [0, 1, 2]
    node.stop()
    node.join(5)
    node.mailbox.put(StartAllreduce(9))  # after stop: dropped, no write into a closed pipe
    time.sleep(0.05)
    assert len(rec.got) == 3


def test_large_payloads_both_ways_from_handlers_do_not_deadlock():
    """Each node answers every big message with a big message of its own from
    inside its handler.  Its dispatcher is the only thread reading its
    sockets, so a blocking write there could wait for a peer that is itself
    blocked writing back, once both socket buffers are full.  Sends never
    block the handler: what the buffer cannot take goes to a flusher."""
    K, big = 12, 1 << 21  # 8 MiB fp32 per message, well past a socket buffer

    class Pong:
        def __init__(self):
            self.node = None
            self.peer = None
            self.seen = 0
            self.done = threading.Event()

        def receive(self, m):
            self.seen += 1
            if m.round < K:
                self.node.send(self.peer, ScatterBlock(torch.full((big,), float(m.round + 1)), 0, 1, 0, m.round + 1))
            if self.seen >= K // 2:
                self.done.set()

    a, b = Pong(), Pong()
    na, nb = Node(name="a").start(a), Node(name="b").start(b)
    a.node, b.node, a.peer, b.peer = na, nb, nb.address, na.address
    for r in range(4):  # both sides start at once: four big messages in flight each way
        na.send(nb.address, ScatterBlock(torch.zeros(big), 0, 1, 0, 2 * r))
        nb.send(na.address, ScatterBlock(torch.zeros(big), 0, 1, 0, 2 * r))
    assert a.done.wait(60) and b.done.wait(60), (a.seen, b.seen)
    for n in (na, nb):
        n.stop()
        n.join(5)


def _native():
    from akka_allreduce_amd._native_loader import load

    return load()


def test_native_data_frames_interoperate_with_the_python_codec():
    """csrc/runtime/frames.h against wire.py: frames the native outbox builds
    decode in Python to the same messages, and frames Python encodes (every
    integer width msgpack picks, fp32 and bf16, empty and long values) parse
    natively to the same fields; other messages are never taken natively."""
    import numpy as np

    from akka_allreduce_amd.messages import ReduceBlock

    n = _native()
    rng = np.random.default_rng(0)
    for kind in (1, 2):
        for nvals in (0, 1, 3, 70, 20000):
            for dtype in ("float32", "bfloat16"):
                for ints in ((0, 1, 2, 3, 4), (127, 128, 255, 256, 65535), (65536, 2**31 - 1, 7, 300, 2**20)):
                    src, dest, chunk, rnd, cnt = ints
                    es = 4 if dtype == "float32" else 2
                    val = rng.integers(0, 255, nvals * es, dtype=np.uint8).tobytes()
                    frame = n.frame_encode(kind, val, dtype, src, dest, chunk, rnd, cnt)
                    body = frame[4:]
                    assert int.from_bytes(frame[:4], "big") == len(body)
                    m = wire.decode(body, lambda a: None)
                    assert type(m) is (ScatterBlock if kind == 1 else ReduceBlock)
                    assert (m.srcId, m.destId, m.chunkId, m.round) == (src, dest, chunk, rnd)
                    assert wire._tensor_bytes(m.value) == (val, dtype)
                    if kind == 2:
                        assert m.count == cnt
                    # and back: Python's encoding parses natively
                    t = m.value
                    py = (ScatterBlock(t, src, dest, chunk, rnd) if kind == 1
                          else ReduceBlock(t, src, dest, chunk, rnd, cnt))
                    pb = wire.encode(py, lambda r: None)[4:]
                    d = n.frame_parse(pb)
                    assert d is not None and d["kind"] == kind and d["value"] == val and d["dtype"] == dtype
                    assert (d["src"], d["dest"], d["chunk"], d["round"]) == (src, dest, chunk, rnd)
                    if kind == 2:
                        assert d["count"] == cnt
    for other in (StartAllreduce(5),):
        assert n.frame_parse(wire.encode(other, lambda r: None)[4:]) is None
    assert n.frame_parse(b"\x87") is None and n.frame_parse(b"") is None  # truncated: not taken


def test_native_splitter_keeps_frame_order_across_cuts():
    """FrameSplitter (the native path of a worker's connections): frames cut
    anywhere across recvs come out whole and in order; with no worker core
    every frame is handed back (nothing is applied natively)."""
    n = _native()
    frames = [wire.encode(StartAllreduce(r), lambda ref: None) for r in range(3)]
    frames.append(wire.encode(ScatterBlock(torch.arange(5, dtype=torch.float32), 0, 1, 2, 3), lambda ref: None))
    frames.append(wire.encode(StartAllreduce(9), lambda ref: None))
    blob = b"".join(frames)
    for cuts in ((1,), (4, 5), (7, 30, 31), tuple(range(1, len(blob)))):
        sp = n.FrameSplitter()
        got, last = [], 0
        for c in cuts + (len(blob),):
            sp.append(blob[last:c])
            last = c
            while True:
                body = sp.run(None)
                if body is None:
                    break
                got.append(wire.decode(body, lambda a: None))
        assert [type(m).__name__ for m in got] == ["StartAllreduce"] * 3 + ["ScatterBlock", "StartAllreduce"]
        assert [m.round for m in got] == [0, 1, 2, 3, 9] and sp.pending == 0


def test_native_splitter_large_frames_and_compaction():
    """Frames larger than a recv, fed in 4 KiB pieces, across the splitter's
    buffer compaction (it drops consumed bytes once they pass 64 KiB): every
    payload comes out intact and in order."""
    n = _native()
    frames = [wire.encode(ScatterBlock(torch.full((50_000 + r,), float(r)), 0, 1, r, r), lambda ref: None)
              for r in range(12)]
    blob = b"".join(frames)
    sp = n.FrameSplitter()
    got = []
    for i in range(0, len(blob), 4096):
        sp.append(blob[i:i + 4096])
        while True:
            body = sp.run(None)
            if body is None:
                break
            got.append(wire.decode(body, lambda a: None))
    assert [m.round for m in got] == list(range(12)) and sp.pending == 0
    for r, m in enumerate(got):
        assert m.value.numel() == 50_000 + r and bool((m.value == float(r)).all())


def test_native_splitter_refuses_an_oversized_frame():
    """A length prefix past the frame limit is a corrupt stream: ValueError
    (the runtime closes the connection), never a frame handed on."""
    import pytest

    sp = _native().FrameSplitter()
    sp.append(b"\xff\xff\xff\xff" + b"x" * 16)
    with pytest.raises(ValueError):
        sp.run(None)
