"""Configuration: the reference's programmatic config types plus a file config.

* ``ThresholdConfig``, ``DataConfig``, ``WorkerConfig`` mirror
  ``AllreduceMaster.scala:148-150`` (same field names).
* ``AppConfig`` replaces the Akka/HOCON ``application.conf`` (CONF:1-34):
  control-plane address, failure-detector timings, logging, and -- unlike the
  reference, whose README says thresholds are "hardcoded in AllreduceMaster"
  (README.md:5) -- the allreduce parameters themselves.  Loaded from YAML or
  JSON (``yaml.safe_load``), then overridden by ``AKKA_*`` environment
  variables, then by explicit keyword overrides.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, Optional

import yaml


@dataclass
class ThresholdConfig:
    thAllreduce: float = 1.0  # "online nodes" threshold: fraction of workers that must complete a round
    thReduce: float = 1.0     # "scatter" threshold: fraction of scattered copies needed to reduce a chunk
    thComplete: float = 1.0   # "reduce" threshold: fraction of reduced chunks needed to complete a round

    def validate(self) -> None:
        for k in ("thAllreduce", "thReduce", "thComplete"):
            v = getattr(self, k)
            if not (0.0 < float(v) <= 1.0):
                raise ValueError(f"{k} must be in (0, 1], got {v}")


@dataclass
class DataConfig:
    dataSize: int = 10
    maxChunkSize: int = 2
    maxRound: int = 100

    def validate(self) -> None:
        if self.dataSize < 0:
            raise ValueError("dataSize must be >= 0")
        if self.maxChunkSize < 1:
            raise ValueError("maxChunkSize must be >= 1")


@dataclass
class WorkerConfig:
    totalSize: int = 2
    maxLag: int = 1

    def validate(self) -> None:
        if self.totalSize < 1:
            raise ValueError("totalSize must be >= 1")
        if self.maxLag < 0:
            raise ValueError("maxLag must be >= 0")


@dataclass
class ClusterSettings:
    host: str = "127.0.0.1"
    port: int = 2551
    # Failure detection (CONF:18-20: auto-down-unreachable-after = 10s)
    heartbeat_interval_s: float = 1.0
    unreachable_after_s: float = 10.0
    registration_timeout_s: float = 5.0  # M:26
    # Cluster metrics (CONF:26-34): node sample attached to a heartbeat this often (0: off)
    metrics_interval_s: float = 10.0


@dataclass
class EngineSettings:
    device: str = "auto"          # "auto" | "cpu" | "cuda" | "cuda:N"
    dtype: str = "float32"        # "float32" | "bfloat16"
    transport: str = "auto"       # "auto" | "rccl" | "tcp"
    broadcast_lag: int = 2        # pipeline distance between a chunk's scatter and broadcast steps
    reduce_impl: str = "auto"     # gfx950 reduce kernel: auto | vec | lds


@dataclass
class AppConfig:
    cluster: ClusterSettings = field(default_factory=ClusterSettings)
    thresholds: ThresholdConfig = field(default_factory=ThresholdConfig)
    data: DataConfig = field(default_factory=DataConfig)
    workers: WorkerConfig = field(default_factory=WorkerConfig)
    engine: EngineSettings = field(default_factory=EngineSettings)
    log_level: str = "INFO"       # CONF:22
    checkpoint: int = 50          # throughput print interval in rounds (W:317)

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)


_SECTIONS = {
    "cluster": ClusterSettings,
    "thresholds": ThresholdConfig,
    "data": DataConfig,
    "workers": WorkerConfig,
    "engine": EngineSettings,
}


def _coerce(cur: Any, val: Any) -> Any:
    if isinstance(cur, bool):
        return str(val).lower() in ("1", "true", "yes", "on") if isinstance(val, str) else bool(val)
    if isinstance(cur, int) and not isinstance(cur, bool):
        return int(val)
    if isinstance(cur, float):
        return float(val)
    return val


def _apply(cfg: AppConfig, d: Dict[str, Any]) -> None:
    for k, v in d.items():
        if k in _SECTIONS and isinstance(v, dict):
            sec = getattr(cfg, k)
            for sk, sv in v.items():
                if not hasattr(sec, sk):
                    raise KeyError(f"unknown config key {k}.{sk}")
                setattr(sec, sk, _coerce(getattr(sec, sk), sv))
        elif hasattr(cfg, k) and k not in _SECTIONS:
            setattr(cfg, k, _coerce(getattr(cfg, k), v))
        else:
            raise KeyError(f"unknown config key {k}")


def default_config_path() -> str:
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return os.path.join(here, "conf", "application.yaml")


def load_config(path: Optional[str] = None, env: Optional[Dict[str, str]] = None, **overrides: Any) -> AppConfig:
    """Load file config (YAML/JSON), then ``AKKA_<SECTION>_<KEY>`` env vars, then overrides.

    Overrides use ``section__key=value`` (e.g. ``thresholds__thReduce=0.75``).
    """
    cfg = AppConfig()
    path = path if path is not None else os.environ.get("AKKA_CONFIG", default_config_path())
    if path and os.path.exists(path):
        with open(path) as f:
            text = f.read()
        d = json.loads(text) if path.endswith(".json") else yaml.safe_load(text)
        if d:
            _apply(cfg, d)
    env = os.environ if env is None else env
    for sec_name, sec_cls in _SECTIONS.items():
        sec = getattr(cfg, sec_name)
        for f_ in dataclasses.fields(sec_cls):
            key = f"AKKA_{sec_name.upper()}_{f_.name.upper()}"
            if key in env:
                setattr(sec, f_.name, _coerce(getattr(sec, f_.name), env[key]))
    if "AKKA_LOG_LEVEL" in env:
        cfg.log_level = env["AKKA_LOG_LEVEL"]
    for k, v in overrides.items():
        if "__" in k:
            sec, key = k.split("__", 1)
            _apply(cfg, {sec: {key: v}})
        else:
            _apply(cfg, {k: v})
    cfg.thresholds.validate()
    cfg.data.validate()
    cfg.workers.validate()
    return cfg
