"""Master-driven cluster with several GPU workers on one MI355X: the master's
InitWorkers carries the data-plane description and every worker brings its
transport up from it (the path RCCL takes with a unique id, here with the
in-process loopback hubs), then the master paces rounds to maxRound
(AllreduceMaster M:36-63, worker InitWorkers W:35-90).  Each worker is an
actor on its own thread (one mailbox, one message at a time); the reactive
workers poll their in-flight transfers between messages."""
import queue
import threading

import pytest
import torch

from akka_allreduce_amd import AllreduceMaster, AllreduceWorker
from akka_allreduce_amd.messages import InitWorkers

pytestmark = pytest.mark.gpu


class ThreadActor:
    def __init__(self, actor, poll=False):
        self.actor = actor
        self.q = queue.Queue()
        self.poll = poll
        self.errors = []
        self.stop = False
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def tell(self, msg, sender=None):
        self.q.put(msg)

    def _run(self):
        while not self.stop:
            try:
                msg = self.q.get(timeout=0.0005 if self.poll else 0.05)
            except queue.Empty:
                if self.poll and getattr(self.actor, "initialized", False):
                    try:
                        self.actor.poll()
                    except Exception as e:  # pragma: no cover
                        self.errors.append(e)
                continue
            try:
                if callable(msg):  # run on this actor's thread (e.g. the master's MemberUp)
                    msg()
                else:
                    self.actor.receive(msg)
            except Exception as e:  # pragma: no cover - surfaced by the test
                self.errors.append(e)


@pytest.mark.parametrize("transport,n", [("stream", 2), ("stream", 4), ("reactive", 3)])
def test_master_brings_up_gpu_workers_transport(native, transport, n):
    dev = torch.device("cuda", 0)
    S, C, rounds = (1 << 16) + 3, 4096, 12
    hub = native.LoopbackHub(n) if transport == "stream" else native.PairLoopbackHub(n)
    kind = "loopback" if transport == "stream" else "loopback_pair"
    outs = {i: [] for i in range(n)}
    done = threading.Event()

    def source(i):
        return lambda req: torch.full((S,), float(i + 1), device=dev) + req.iteration

    def sink(i):
        def f(o):
            o.wait()
            outs[i].append((o.iteration, o.data.clone(), o.count.clone()))
        return f

    master = AllreduceMaster(n, 1.0, 1.0, 1.0, 2, S, rounds - 1, C, on_finished=done.set)
    mref = ThreadActor(master)
    workers = [AllreduceWorker(source(i), sink(i), device=dev, transport=transport, strict=True, name=f"g{i}")
               for i in range(n)]
    for w in workers:
        w.reactive_timeout = 60.0
    refs = [ThreadActor(w, poll=transport == "reactive") for w in workers]

    def init(ids):  # the master's InitWorkers, with the data plane to bring up and the master's mailbox
        for idx in ids:
            m = InitWorkers(dict(master.workers), n, mref, idx, 1.0, 1.0, 2, S, C)
            m.transport = {"kind": kind, "hub": hub}
            master.workers[idx].tell(m)

    master._init_workers = init
    try:
        for r in refs:  # MemberUp on the master's own thread (M:36-44)
            mref.tell(lambda r=r: master.member_up(r))
        assert done.wait(120), f"master stuck at round {master.round}"
        for r in refs + [mref]:
            r.stop = True
            r.t.join(timeout=30)
        assert not any(r.errors for r in refs + [mref]), [r.errors for r in refs + [mref]]
        torch.cuda.synchronize()
        want_base = float(sum(range(1, n + 1)))
        for i in range(n):
            its = [it for it, _, _ in outs[i]]
            assert its[:rounds] == list(range(rounds)), its
            for it, data, count in outs[i]:
                assert torch.equal(data, torch.full_like(data, want_base + n * it)), (i, it)
                assert bool((count == n).all())
        for w in workers:
            assert w.transport_spec[0] == kind and w.state()["round"] >= rounds
    finally:
        for r in refs:
            r.stop = True
        hub_release = getattr(hub, "release_all", None)
        if hub_release:
            hub_release()
        for w in workers:
            w.close()
