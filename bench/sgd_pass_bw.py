"""The config-5 fused average + SGD + bf16 shadow pass alone (count_mean
kernel, 41.7 M fp32 parameters = the MLP's 167 MB, N=1 geometry with 1 M
element chunks): µs per pass and TB/s of the bytes it must move (sum and
parameters read, parameters and shadow written).  AKKA_CM_MAXGRID in the
environment sets the grid.  One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    from akka_allreduce_amd.data import AllReduceOutput, Geometry

    S, N, C = 41_756_136, 1, 1 << 20
    g = Geometry(S, N, C)
    d = torch.randn(S, device="cuda")
    pc = torch.ones((N, g.kmax), device="cuda", dtype=torch.int32)
    y = torch.randn(S, device="cuda")
    sh = torch.empty(S, device="cuda", dtype=torch.bfloat16)
    out = AllReduceOutput(d, counts_per_chunk=pc, geometry=g)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        out.axpy_mean_(y, -1e-6, shadow=sh)
    torch.cuda.synchronize()
    a.record()
    for _ in range(30):
        out.axpy_mean_(y, -1e-6, shadow=sh)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / 30 * 1e3
    print(json.dumps({"maxgrid": os.environ.get("AKKA_CM_MAXGRID", "default"), "us": round(us, 1),
                      "TBps": round((3 * 4 + 2) * S / us / 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
