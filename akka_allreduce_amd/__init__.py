"""akka_allreduce_amd: MI355X-native threshold (straggler-tolerant) allreduce.

Capabilities of GuixingLin/akka-allreduce, re-designed for AMD Instinct MI355X:
per-GPU worker ranks exchanging chunks over xGMI with RCCL point-to-point,
gfx950 HIP kernels for the chunk sums, a native C++ round engine, and a
host-side master for membership and round pacing.
"""
from .config import AppConfig, DataConfig, ThresholdConfig, WorkerConfig, load_config
from .data import AllReduceInput, AllReduceInputRequest, AllReduceOutput, Geometry
from .messages import (
    CompleteAllreduce,
    Heartbeat,
    InitWorkers,
    ReduceBlock,
    RegisterWorker,
    ScatterBlock,
    Shutdown,
    StartAllreduce,
    WorkerTerminated,
)
from .worker import AllreduceWorker
from .master import AllreduceMaster

__all__ = [
    "AllreduceMaster",
    "AllreduceWorker",
    "AllReduceInput",
    "AllReduceInputRequest",
    "AllReduceOutput",
    "AppConfig",
    "CompleteAllreduce",
    "DataConfig",
    "Geometry",
    "Heartbeat",
    "InitWorkers",
    "ReduceBlock",
    "RegisterWorker",
    "ScatterBlock",
    "Shutdown",
    "StartAllreduce",
    "ThresholdConfig",
    "WorkerConfig",
    "WorkerTerminated",
    "load_config",
]

__version__ = "0.1.0"
