"""N=1 round = one local pass input -> output.  Compare our NSRC=1 reduce
kernel (the round's actual path) with torch's copy_ (hipMemcpyAsync D2D blit)
at the headline and config-3 sizes.  Prints one JSON line per case."""
import json
import time

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from akka_allreduce_amd._native_loader import load  # noqa: E402


def t_of(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    n = load()
    s = torch.cuda.current_stream().cuda_stream
    for mib, dt in ((256, torch.float32), (1024, torch.bfloat16), (1024, torch.float32)):
        S = (mib << 20) // torch.tensor([], dtype=dt).element_size()
        a = torch.randn(S, device="cuda").to(dt)
        b = torch.empty_like(a)
        name = "float32" if dt == torch.float32 else "bfloat16"
        res = {"MiB": mib, "dtype": name}
        for impl in ("auto", "vec_nts", "vec", "vec_both"):
            try:
                f = lambda: n.reduce(b.data_ptr(), [a.data_ptr()], S, name, s, impl)  # noqa: E731
                dt_s = t_of(f)
                res[f"kernel_{impl}_TBps"] = round(2 * a.numel() * a.element_size() / dt_s / 1e12, 3)
            except Exception as e:  # noqa: BLE001
                res[f"kernel_{impl}_err"] = str(e)[:80]
        dt_s = t_of(lambda: b.copy_(a))
        res["torch_copy_TBps"] = round(2 * a.numel() * a.element_size() / dt_s / 1e12, 3)
        assert torch.equal(a, b)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
