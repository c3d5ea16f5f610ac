"""Master/worker cluster flow with a GPU worker (one MI355X): the master mints
the RCCL id for an all-GPU cluster, the worker's data plane runs on cuda:0
(N=1: local rounds, no RCCL needed), the demo sink checks exactness and the
master paces rounds to maxRound -- the reference's startUp flow end to end."""
import pytest
import torch

from akka_allreduce_amd.config import DataConfig, ThresholdConfig, WorkerConfig
from akka_allreduce_amd.parallel.cluster import start_master, start_worker

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("size,chunk", [(10, 2), (778, 3), (1 << 20, 1 << 16)])
def test_master_with_gpu_worker(size, chunk):
    m = start_master(ThresholdConfig(1.0, 1.0, 1.0), DataConfig(size, chunk, 30), WorkerConfig(1, 2), port=0,
                     transport="auto", unreachable_after_s=30.0)
    w = start_worker(m.address, size, checkpoint=5, assert_multiple=1, device="cuda:0", printer=lambda *_: None)
    try:
        assert m.wait(60), f"master stuck at round {m.master.round}"
        assert w.wait(20)
        sink = w.worker.dataSink
        assert sink.failures == 0 and sink.rounds >= 30
        assert w.worker.device.type == "cuda"
    finally:
        m.stop()
        w.stop()
    torch.cuda.synchronize()


def test_node_metrics_gpu_sample():
    """amdsmi side of the cluster metrics: one entry per visible GPU; sampling never raises."""
    from akka_allreduce_amd.utils.node_metrics import sample

    torch.ones(1 << 20, device="cuda").sum().item()
    s = sample()
    assert s["mem_total_mb"] > 0
    print("node metrics sample:", s)
    if s["gpus"]:  # amdsmi present on the box
        assert all(isinstance(g, dict) for g in s["gpus"])
        assert any(g for g in s["gpus"]), "amdsmi handles found but no counter readable"
