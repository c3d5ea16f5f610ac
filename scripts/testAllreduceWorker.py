#!/usr/bin/env python3
"""Port of scripts/testAllreduceWorker.sc: a worker with dataSize 778, checkpoint 10,
assertMultiple 4 (exactness check against 4 x input; reference scripts/testAllreduceWorker.sc:4).
Start four of these after testAllreduceMaster.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from akka_allreduce_amd.parallel.cluster import start_worker  # noqa: E402

if __name__ == "__main__":
    master = os.environ.get("MASTER", "127.0.0.1:2551")
    w = start_worker(master, 778, checkpoint=10, assert_multiple=4, device=os.environ.get("DEVICE", "cpu"))
    w.wait()
    sys.exit(1 if w.worker.dataSink.failures else 0)
