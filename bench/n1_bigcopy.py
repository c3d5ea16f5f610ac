"""The N=1 round of BASELINE config 3 (1 GiB bf16) is a one-source reduce
pass, i.e. a streamed copy well beyond the 256 MiB Infinity Cache.  Times
chunk_reduce([x]) per impl (AKKA_VEC_BPC in the environment sets the
blocks per CU) against torch's copy_.  One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    from akka_allreduce_amd.ops import chunk_reduce

    nbytes = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
    dtype = torch.bfloat16 if (len(sys.argv) <= 2 or sys.argv[2] == "bf16") else torch.float32
    x = torch.randn(nbytes // 4, device="cuda").view(dtype)
    out = torch.empty_like(x)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def t(fn, iters=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / iters * 1e3

    res = {"bytes": nbytes, "dtype": str(dtype), "bpc": os.environ.get("AKKA_VEC_BPC", "auto")}
    for impl in ("auto", "vec_nts", "vec_ntl", "vec_both"):
        us = t(lambda: chunk_reduce([x], out=out, impl=impl))
        res[impl] = {"us": round(us, 1), "copy_TBps": round(2 * nbytes / us / 1e6, 3)}
    us = t(lambda: out.copy_(x))
    res["torch_copy"] = {"us": round(us, 1), "copy_TBps": round(2 * nbytes / us / 1e6, 3)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
