"""Worker process for tests/test_cluster_onesided*.py: one AllreduceWorker on
the one-sided lane (``--transport onesided``) joining a master, contributing
2^id every round so each output chunk encodes its contributor set; an
optional straggler sleeps ``--delay-ms`` in its data source (W:197-204).
Writes <out-dir>/worker<pid>.json at Shutdown: the sink's per-round record
(round, arrival time, contributor-set check) and the lane's counters."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--master", required=True)
    ap.add_argument("--size", type=int, required=True)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--delay-ms", type=float, default=0.0)
    ap.add_argument("--out-dir", required=True)
    ap.add_argument("--timeout-s", type=float, default=240.0)
    ap.add_argument("--die-after", type=int, default=-1, help="exit abruptly once this round reached the sink")
    ap.add_argument("--compute-ms", type=float, default=0.0, help="every round's data source sleeps this long")
    ap.add_argument("--progress-file", default="", help="the sink writes the last round it got here")
    a = ap.parse_args()
    import faulthandler
    import logging

    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    faulthandler.dump_traceback_later(max(10.0, a.timeout_s - 5), exit=False)  # stacks into the log on a hang
    from akka_allreduce_amd.parallel.cluster import start_worker

    holder = {}
    recs = []
    src_t = []

    def source(req):
        src_t.append(time.perf_counter())
        if a.delay_ms or a.compute_ms:
            time.sleep((a.delay_ms + a.compute_ms) / 1e3)
        wid = holder["w"].worker.id
        return torch.full((a.size,), float(1 << wid))

    kept = []

    def sink(o):
        # cheap in the round path: keep the output, check after the job
        kept.append((int(o.iteration), o.data.float().cpu(),
                     o.counts_per_chunk.cpu() if o.counts_per_chunk is not None else None, o.geometry))
        recs.append({"round": int(o.iteration), "t": time.perf_counter(), "t_src": src_t[-1] if src_t else 0.0})
        if a.progress_file:
            with open(a.progress_file + ".tmp", "w") as f:
                f.write(str(int(o.iteration)))
            os.replace(a.progress_file + ".tmp", a.progress_file)
        if 0 <= a.die_after <= int(o.iteration):
            os._exit(0)  # abrupt: no Shutdown, no retire -- the master's failure detector must notice

    def check(rec, item):
        _, data, cpc, g = item
        bad = 0
        if cpc is not None and g is not None:
            for p in range(g.workerNum):
                for k in range(g.num_chunks(p)):
                    s, e = g.chunk_range(p, k)
                    seg = data[s:e]
                    v = float(seg[0])
                    c = int(cpc[p, k])
                    if not bool((seg == v).all()) or v != int(v) or bin(int(v)).count("1") != c:
                        bad += 1
            n = sum(g.num_chunks(p) for p in range(g.workerNum))
            rec["mean_count"] = float(sum(int(cpc[p, k]) for p in range(g.workerNum)
                                          for k in range(g.num_chunks(p)))) / max(1, n)
            rec["block_counts"] = [int(cpc[p, 0]) if g.num_chunks(p) else 0 for p in range(g.workerNum)]
            # per worker id: chunks whose contributor set includes it
            rec["with"] = [sum((int(float(data[g.chunk_range(p, k)[0]])) >> q) & 1 for p in range(g.workerNum)
                               for k in range(g.num_chunks(p)) if g.chunk_range(p, k)[1] > g.chunk_range(p, k)[0])
                           for q in range(g.workerNum)]
            rec["chunks"] = n
        else:
            rec["mean_count"] = 0.0
            rec["block_counts"] = None  # a round force-completed by catch-up: zeros, count 0 (W:100-106)
        rec["bad"] = bad

    dev = a.device
    w = start_worker(a.master, a.size, device=dev, data_source=source, data_sink=sink, transport="onesided",
                     printer=lambda *x: None)
    holder["w"] = w
    done = w.wait(a.timeout_s)
    for rec, item in zip(recs, kept):
        check(rec, item)
    wk = w.worker
    res = {"id": wk.id, "straggler": a.delay_ms > 0, "records": recs, "errors": [repr(e) for e in wk.errors],
           "forced_rounds": wk.forced_rounds, "finished": bool(done),
           "stats": wk.ar.stats() if wk.ar is not None else None}
    with open(os.path.join(a.out_dir, f"worker{os.getpid()}.json"), "w") as f:
        json.dump(res, f)
    w.stop()
    os._exit(0)  # the lane's windows go with the process


if __name__ == "__main__":
    main()
