"""Diagnose tests/test_dp_ipc_gpu.py: N ranks (one card) run the DP-SGD loop
on the ipc data plane and save every round's input and output; rank 0 then
checks out == sum of the ranks' inputs per block and reports where it is not.
Run under torch.distributed.run; AKKA_DIAG_MODE = pull | bcast | fused."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out_dir = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from akka_allreduce_amd.models.mlp import MLP, dp_sgd_step, synthetic_batch
    from akka_allreduce_amd.parallel import ThresholdAllreduce
    from akka_allreduce_amd.parallel.dp import GradientBucket

    torch.manual_seed(0)
    model = MLP(256, 512, 10).to(dev)
    bucket = GradientBucket(list(model.parameters()), flatten_params=True)
    ar = ThresholdAllreduce(bucket.numel, max_chunk_size=1 << 14, device=dev, data_plane="ipc")
    mode = os.environ.get("AKKA_DIAG_MODE", "pull")
    ar.set_ipc_mode("bcast" if "bcast" in mode else "pull", fused="fused" in mode)
    sync_each = os.environ.get("AKKA_DIAG_SYNC") == "1"
    rec = []

    def recording_ar(x):
        xin = x.detach().clone()
        o = ar(x)
        if sync_each:
            torch.cuda.synchronize()
        rec.append((xin, o.data.detach().clone(), o.counts_per_chunk.detach().clone()))  # o.count would disable the fused update
        return o

    for s in range(steps):
        g = torch.Generator(device=dev).manual_seed(100 * s + rank)
        x, y = synthetic_batch(64, 256, 10, device=dev, generator=g)
        dp_sgd_step(model, x, y, 0.1, recording_ar, bucket)
    torch.cuda.synchronize()
    flat = torch.cat([p.detach().reshape(-1).float().cpu() for p in model.parameters()])
    torch.save({"rec": [(a.cpu(), b.cpu(), c.cpu()) for a, b, c in rec], "err": ar.ipc_error(),
                "S": bucket.numel, "flat": flat}, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    if rank == 0:
        allr = [torch.load(os.path.join(out_dir, f"r{i}.pt"), weights_only=True) for i in range(world)]
        S = allr[0]["S"]
        step = -(-S // world)
        for s in range(steps):
            want = sum(allr[i]["rec"][s][0].double() for i in range(world)).float()
            for i in range(world):
                o = allr[i]["rec"][s][1]
                bad = (o - want).abs() > 1e-6 * (1 + want.abs())
                msg = []
                for b in range(world):
                    sl = slice(b * step, min(S, (b + 1) * step))
                    nb = int(bad[sl].sum())
                    if nb:
                        # is it an earlier round's value (stale) of some rank's contribution?
                        stale = ""
                        if s > 0:
                            prev = sum(allr[k]["rec"][s - 1][0].double() for k in range(world)).float()
                            stale = f" eq_prev_sum={int(((o[sl] - prev[sl]).abs() <= 1e-6 * (1 + prev[sl].abs())).sum())}"
                            for k in range(world):
                                alt = want.clone()
                                alt = alt - allr[k]["rec"][s][0] + allr[k]["rec"][s - 1][0]
                                stale += f" stale_r{k}={int(((o[sl] - alt[sl]).abs() <= 1e-5 * (1 + alt[sl].abs())).sum())}"
                        msg.append(f"block{b}: {nb}/{sl.stop - sl.start} bad{stale}")
                cnt = allr[i]["rec"][s][2]
                print(f"step {s} rank {i}: {'OK' if not msg else '; '.join(msg)} err={allr[i]['err']} "
                      f"counts min/max={int(cnt.min())}/{int(cnt.max())}", flush=True)
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
        from test_dp_ipc_gpu import _reference

        want = _reference(world, steps, dev)
        for i in range(world):
            d = (allr[i]["flat"] - want).abs()
            print(f"final rank {i}: max|diff| vs reference {float(d.max()):.3g}, n>1e-5: {int((d > 1e-5).sum())}, "
                  f"equal to rank0: {torch.equal(allr[i]['flat'], allr[0]['flat'])}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
