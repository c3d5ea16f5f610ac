#!/usr/bin/env python3
"""Port of scripts/testAllreduceMaster.sc: 4 workers, dataSize 778, maxChunkSize 3,
maxRound 1000, maxLag 3, all thresholds 1.0 (reference scripts/testAllreduceMaster.sc:7-24)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_amd.config import DataConfig, ThresholdConfig, WorkerConfig  # noqa: E402
from akka_allreduce_amd.parallel.cluster import start_master  # noqa: E402

if __name__ == "__main__":
    m = start_master(ThresholdConfig(thAllreduce=1.0, thReduce=1.0, thComplete=1.0),
                     DataConfig(dataSize=778, maxChunkSize=3, maxRound=int(os.environ.get("MAX_ROUND", 1000))),
                     WorkerConfig(totalSize=4, maxLag=3), port=int(os.environ.get("PORT", 2551)))
    print(f"master on {m.address}", flush=True)
    m.wait()
    m.stop()
