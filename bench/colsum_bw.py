"""Bias-gradient column sum (ops/colsum.py) on one GPU: the gfx950 kernel's
variants (row splits, write-through vs fenced hand-off of the partial rows)
against torch.sum, alone and right behind the fp32-out dW GEMM that precedes
it in the MLP backward (L2 full of dirty lines).  One JSON line per case.

    python bench/colsum_bw.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    from akka_allreduce_amd.ops import colsum

    dev = torch.device("cuda", 0)

    def t_us(fn, iters=200):
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / iters * 1e3

    for M, N, K in ((256, 8192, 4096), (256, 1000, 8192)):
        g = torch.randn(M, N, device=dev).to(torch.bfloat16)
        xin = torch.randn(M, K, device=dev).to(torch.bfloat16)
        gw = torch.empty(N, K, device=dev)
        out = torch.empty(N, device=dev)
        gemm = lambda: torch.mm(g.t(), xin, out_dtype=torch.float32, out=gw)  # noqa: E731
        variants = {"torch_sum": lambda: torch.sum(g, 0, dtype=torch.float32, out=out),
                    "lite_auto": lambda: colsum(g, out=out),
                    "fenced_auto": lambda: colsum(g, out=out, lite=False)}
        for sp in (1, 2, 4, 8, 16):
            variants[f"lite_s{sp}"] = (lambda sp=sp: colsum(g, out=out, splits=sp))
        want = g.float().sum(0)
        t_gemm = t_us(gemm, 50)
        for name, fn in variants.items():
            fn()
            torch.cuda.synchronize()
            err = float((out - want).abs().max())
            alone = t_us(fn)
            behind = t_us(lambda: (gemm(), fn()), 50) - t_gemm
            print(json.dumps({"M": M, "N": N, "variant": name, "us_alone": round(alone, 2),
                              "us_behind_gemm": round(behind, 2), "gemm_us": round(t_gemm, 2),
                              "max_err": err}), flush=True)


if __name__ == "__main__":
    main()
