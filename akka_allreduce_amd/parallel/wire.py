"""Wire codec for the control plane (and the CPU data plane).

Replaces Akka remoting's Java serialization of the case classes.
Frames are ``[u32 big-endian length][msgpack map]``; msgpack carries only
plain data (no code is ever deserialised).  Actor references travel as
``"host:port"`` addresses and are turned back into references by the
receiving runtime.  Tensor payloads (CPU-cluster ScatterBlock/ReduceBlock)
travel as raw little-endian bytes plus a dtype tag.
"""
from __future__ import annotations

import struct
from typing import Any, Callable, Dict, Optional

import msgpack
import torch

from ..messages import (
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

_HDR = struct.Struct(">I")
MAX_FRAME = 1 << 31

_DT = {torch.float32: "float32", torch.bfloat16: "bfloat16"}
_DT_INV = {v: k for k, v in _DT.items()}


def _tensor_bytes(v: Any) -> tuple[bytes, str]:
    # fast path: a contiguous CPU tensor of a wire dtype (every engine payload
    # is one) -- each torch call below costs microseconds, a round of the
    # reference's demo (10 floats, 2-float chunks) sends ~7 of these per worker
    if isinstance(v, torch.Tensor) and v.device.type == "cpu" and not v.requires_grad and v.is_contiguous():
        if v.dtype == torch.float32:
            return v.numpy().tobytes(), "float32"
        if v.dtype == torch.bfloat16:
            return v.view(torch.int16).numpy().tobytes(), "bfloat16"
    t = v if isinstance(v, torch.Tensor) else torch.as_tensor(v, dtype=torch.float32)
    t = t.detach().reshape(-1).contiguous().cpu()
    if t.dtype not in _DT:
        t = t.float()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().tobytes(), "bfloat16"
    return t.numpy().tobytes(), _DT[t.dtype]


def _bytes_tensor(b: bytes, dt: str) -> torch.Tensor:
    if not b:  # (torch.frombuffer refuses an empty buffer)
        return torch.empty(0, dtype=_DT_INV[dt])
    if dt == "bfloat16":
        return torch.frombuffer(bytearray(b), dtype=torch.int16).view(torch.bfloat16)
    return torch.frombuffer(bytearray(b), dtype=_DT_INV[dt])


def encode(msg: Any, ref_to_addr: Callable[[Any], Optional[str]]) -> bytes:
    if isinstance(msg, InitWorkers):
        d: Dict[str, Any] = {
            "t": "InitWorkers",
            "workers": {int(k): ref_to_addr(v) for k, v in msg.workers.items()},
            "workerNum": msg.workerNum, "master": ref_to_addr(msg.master), "destId": msg.destId,
            "thReduce": float(msg.thReduce), "thComplete": float(msg.thComplete), "maxLag": msg.maxLag,
            "dataSize": msg.dataSize, "maxChunkSize": msg.maxChunkSize,
            "transport": getattr(msg, "transport", None),
        }
    elif isinstance(msg, StartAllreduce):
        d = {"t": "StartAllreduce", "round": msg.round}
    elif isinstance(msg, ScatterBlock):
        b, dt = _tensor_bytes(msg.value)
        d = {"t": "ScatterBlock", "value": b, "dtype": dt, "srcId": msg.srcId, "destId": msg.destId,
             "chunkId": msg.chunkId, "round": msg.round}
    elif isinstance(msg, ReduceBlock):
        b, dt = _tensor_bytes(msg.value)
        d = {"t": "ReduceBlock", "value": b, "dtype": dt, "srcId": msg.srcId, "destId": msg.destId,
             "chunkId": msg.chunkId, "round": msg.round, "count": msg.count}
    elif isinstance(msg, CompleteAllreduce):
        d = {"t": "CompleteAllreduce", "srcId": msg.srcId, "round": msg.round}
    elif isinstance(msg, RegisterWorker):
        d = {"t": "RegisterWorker", "address": msg.address, "device": msg.device, "hostname": msg.hostname,
             "meta": msg.meta}
    elif isinstance(msg, WorkerTerminated):
        d = {"t": "WorkerTerminated", "workerId": msg.workerId}
    elif isinstance(msg, Heartbeat):
        d = {"t": "Heartbeat", "srcId": msg.srcId, "round": msg.round, "metrics": msg.metrics}
    elif isinstance(msg, Shutdown):
        d = {"t": "Shutdown", "reason": msg.reason}
    else:
        raise TypeError(f"cannot encode {type(msg).__name__}")
    body = msgpack.packb(d, use_bin_type=True)
    return _HDR.pack(len(body)) + body


def decode(body: bytes, addr_to_ref: Callable[[Optional[str]], Any]) -> Any:
    d = msgpack.unpackb(body, raw=False, strict_map_key=False)
    t = d.get("t")
    if t == "InitWorkers":
        m = InitWorkers({int(k): addr_to_ref(v) for k, v in d["workers"].items()}, d["workerNum"],
                        addr_to_ref(d["master"]), d["destId"], d["thReduce"], d["thComplete"], d["maxLag"],
                        d["dataSize"], d["maxChunkSize"])
        if d.get("transport") is not None:
            m.transport = d["transport"]  # type: ignore[attr-defined]
        return m
    if t == "StartAllreduce":
        return StartAllreduce(d["round"])
    if t == "ScatterBlock":
        return ScatterBlock(_bytes_tensor(d["value"], d["dtype"]), d["srcId"], d["destId"], d["chunkId"], d["round"])
    if t == "ReduceBlock":
        return ReduceBlock(_bytes_tensor(d["value"], d["dtype"]), d["srcId"], d["destId"], d["chunkId"], d["round"],
                           d["count"])
    if t == "CompleteAllreduce":
        return CompleteAllreduce(d["srcId"], d["round"])
    if t == "RegisterWorker":
        return RegisterWorker(d["address"], d.get("device"), d.get("hostname", ""), d.get("meta") or {})
    if t == "WorkerTerminated":
        return WorkerTerminated(d["workerId"])
    if t == "Heartbeat":
        return Heartbeat(d["srcId"], d["round"], d.get("metrics"))
    if t == "Shutdown":
        return Shutdown(d.get("reason", ""))
    raise ValueError(f"unknown message type {t!r}")


class FrameReader:
    """Frames of one connection: bytes as they arrive -> complete frame
    bodies.  One ``recv`` may hold several frames (a sender's batch,
    ``Node.send_many``) or part of one."""

    def __init__(self):
        self._buf = bytearray()

    def feed(self, chunk: bytes) -> list:
        """Bytes received on the connection -> the bodies of the frames they
        complete."""
        self._buf += chunk
        out = []
        while len(self._buf) >= 4:
            (n,) = _HDR.unpack_from(self._buf, 0)
            if n > MAX_FRAME:
                raise ValueError(f"frame of {n} bytes exceeds limit")
            if len(self._buf) < 4 + n:
                break
            out.append(bytes(self._buf[4:4 + n]))
            del self._buf[:4 + n]
        return out
