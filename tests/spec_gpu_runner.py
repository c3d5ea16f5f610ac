"""Child process of tests/test_onesided_spec_gpu.py (started with
GPU_MAX_HW_QUEUES=16): runs every spec case on the GPU window harness and
writes {case: {"ok": bool, "error": str, "s": seconds}} to argv[1]."""
import json
import os
import sys
import time
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import test_onesided_spec_gpu as sg  # noqa: E402


def main():
    out = sys.argv[1]
    res = {}
    todo = [(name, None) for name in sg.CASES] + [("test_random_orders_match_reference_rules", s) for s in sg.SEEDS]
    todo += [(name, None) for name in sorted(sg.EXTRA)]
    for name, seed in todo:
        key = name if seed is None else f"random_orders_{seed}"
        t0 = time.monotonic()
        try:
            if name in sg.EXTRA:
                sg.EXTRA[name]()
            else:
                sg.run_case(name, sg.WindowSpecHarness, seed=seed)
            res[key] = {"ok": True, "error": "", "s": round(time.monotonic() - t0, 2)}
        except Exception:  # noqa: BLE001 - recorded per case
            res[key] = {"ok": False, "error": traceback.format_exc()[-2500:], "s": round(time.monotonic() - t0, 2)}
        print(f"{key}: {'ok' if res[key]['ok'] else 'FAILED'} in {res[key]['s']} s", flush=True)
        with open(out, "w") as f:  # after every case: a later hang still leaves the earlier results
            json.dump(res, f)


if __name__ == "__main__":
    main()
