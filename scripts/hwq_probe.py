"""Effective hardware-queue count for streams: park k streams on a wait-value
and check a fresh stream still runs.  Prints JSON for a given GPU_MAX_HW_QUEUES."""
import json
import os
import sys

if len(sys.argv) > 1:
    os.environ["GPU_MAX_HW_QUEUES"] = sys.argv[1]
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from akka_allreduce_amd._native_loader import load  # noqa: E402

k = load().hw_queue_probe(40, 300)
print(json.dumps({"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), "first_blocking_parked_streams": k}))
