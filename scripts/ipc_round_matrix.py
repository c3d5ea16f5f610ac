"""Time whole exact ipc rounds for a matrix of (N, size, dtype, phase-2 mode,
lite, threads), N processes sharing the box's GPU (tests/ipc_ranks.py
--time, 10 timed rounds after 3 warm-ups, no exactness check).  One JSON
line per case: the slowest rank's ms per round and the algbw it implies.

    python scripts/ipc_round_matrix.py --cases "4:536870912:bfloat16:fused:1:1024,4:67108864:float32:fused:1:1024"
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", required=True,
                    help="N:size:dtype:mode:lite:threads[:chunk[:async[:pre_size[:pre_rounds[:pre_del]]]]], comma separated")
    ap.add_argument("--env", default="", help="extra environment for every case, K=V;K=V")
    ap.add_argument("--timeout", type=int, default=240)
    a = ap.parse_args()
    for case in a.cases.split(","):
        f = case.split(":")
        n, size, dtype, mode, lite, threads = int(f[0]), int(f[1]), f[2], f[3], f[4], f[5]
        chunk = int(f[6]) if len(f) > 6 else 0
        async_op = len(f) > 7 and f[7] == "1"
        pre = int(f[8]) if len(f) > 8 else 0
        pre_rounds = int(f[9]) if len(f) > 9 else 5
        pre_del = len(f) > 10 and f[10] == "1"
        with tempfile.TemporaryDirectory() as out:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                   "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                   os.path.join(ROOT, "tests", "ipc_ranks.py"), "--out-dir", out, "--size", str(size),
                   "--dtype", dtype, "--rounds", "0", "--time", "--time-mode", mode, "--chunk", str(chunk),
                   "--pre-size", str(pre), "--pre-rounds", str(pre_rounds)] + (["--time-async"] if async_op else []) \
                + (["--pre-del"] if pre_del else [])
            env = dict(os.environ, AKKA_IPC_LITE=lite, AKKA_IPC_THREADS=threads)
            env.update(kv.split("=", 1) for kv in a.env.split(";") if kv)
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout, cwd=ROOT, env=env)
            rows = []
            for i in range(n):
                p = os.path.join(out, f"rank{i}.json")
                if os.path.exists(p):
                    with open(p) as fh:
                        rows.append(json.load(fh))
        line = {"N": n, "size": size, "dtype": dtype, "mode": mode, "lite": lite == "1", "threads": int(threads),
                "chunk": chunk, "async": async_op, "pre_size": pre, "pre_rounds": pre_rounds, "pre_del": pre_del,
                "env": a.env, "rc": r.returncode}
        if r.returncode == 0 and len(rows) == n:
            ms = max(d["ms_per_round"] for d in rows)
            es = 4 if dtype == "float32" else 2
            line.update(ms_per_round=round(ms, 4), algbw_GBps=round(size * es / (ms * 1e-3) / 1e9, 2),
                        ipc_error=max(d["ipc_error"] for d in rows))
        else:
            line["stderr"] = r.stderr[-600:]
        print(json.dumps(line), flush=True)
        if r.returncode != 0:
            break  # no further GPU step after a failure


if __name__ == "__main__":
    main()
