"""Node metrics: the reference's akka-cluster-metrics + Sigar (CONF:26-34,
build.sbt:20,26), MI355X style.

The reference enables cluster metrics but never reads them.  Here a worker can
attach a sample to its heartbeats (``cluster.metrics_interval_s``) and the
master keeps the latest per worker (``MasterProcess.node_metrics``): host CPU
and memory (psutil) and, per visible GPU, busy %, VRAM in use, power and edge
temperature through AMD SMI.  Every source is optional: a missing library or a
counter the driver refuses simply leaves its keys out.
"""
from __future__ import annotations

import threading
from typing import Any, Dict, List, Optional

_lock = threading.Lock()
_smi: Any = None
_smi_handles: Optional[List[Any]] = None


def _gpu_handles() -> List[Any]:
    global _smi, _smi_handles
    with _lock:
        if _smi_handles is None:
            try:
                import amdsmi

                amdsmi.amdsmi_init()
                _smi = amdsmi
                _smi_handles = list(amdsmi.amdsmi_get_processor_handles())
            except Exception:
                _smi_handles = []
        return _smi_handles


def _gpu_sample(h: Any) -> Dict[str, Any]:
    smi = _smi
    g: Dict[str, Any] = {}
    try:
        act = smi.amdsmi_get_gpu_activity(h)
        g["busy_pct"] = act.get("gfx_activity")
    except Exception:
        pass
    try:
        g["vram_used_mb"] = int(smi.amdsmi_get_gpu_memory_usage(h, smi.AmdSmiMemoryType.VRAM)) >> 20
    except Exception:
        pass
    try:
        p = smi.amdsmi_get_power_info(h)
        g["power_w"] = p.get("current_socket_power", p.get("average_socket_power"))
    except Exception:
        pass
    try:
        g["temp_c"] = smi.amdsmi_get_temp_metric(h, smi.AmdSmiTemperatureType.EDGE,
                                                 smi.AmdSmiTemperatureMetric.CURRENT)
    except Exception:
        pass
    return {k: v for k, v in g.items() if v is not None and v != "N/A"}


def sample(gpus: bool = True) -> Dict[str, Any]:
    """One snapshot: {"cpu_pct", "mem_used_mb", "mem_total_mb", "gpus": [...]}."""
    out: Dict[str, Any] = {}
    try:
        import psutil

        out["cpu_pct"] = psutil.cpu_percent(interval=None)
        vm = psutil.virtual_memory()
        out["mem_used_mb"] = int(vm.used) >> 20
        out["mem_total_mb"] = int(vm.total) >> 20
    except Exception:
        pass
    if gpus:
        out["gpus"] = [_gpu_sample(h) for h in _gpu_handles()]
    return out
