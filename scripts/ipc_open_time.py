"""Time ThresholdAllreduce.enable_ipc (window alloc + handle exchange +
hipIpcOpenMemHandle of every peer's window) for a buffer size / dtype, N
processes sharing the card.  Run under torch.distributed.run."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    import faulthandler

    faulthandler.dump_traceback_later(float(os.environ.get("AKKA_DUMP_AFTER_S", "45")), exit=True)
    nbytes, dtype = int(float(sys.argv[1]) * (1 << 20)), sys.argv[2]
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from akka_allreduce_amd.parallel import ThresholdAllreduce

    dt = torch.bfloat16 if dtype == "bfloat16" else torch.float32
    S = nbytes // (2 if dt == torch.bfloat16 else 4)
    ar = ThresholdAllreduce(S, max_chunk_size=1 << 22, dtype=dt, device=dev, data_plane="ipc_p2p")
    dist.barrier()
    t0 = time.perf_counter()
    ar.enable_ipc()
    t1 = time.perf_counter()
    print(f"rank {rank}: windows open after {t1 - t0:.2f} s", file=sys.stderr, flush=True)
    ar.use_lane("ipc")
    x = torch.ones(S, device=dev, dtype=dt)
    o = ar(x)
    torch.cuda.synchronize()
    ok = bool((o.data == dist.get_world_size()).all())
    print(f"rank {rank} {nbytes >> 20} MiB {dtype} mem={os.environ.get('AKKA_IPC_MEM', 'fine')}: "
          f"enable_ipc {t1 - t0:.2f} s, window {ar.state()['link']['ipc'].get('window_bytes', 0) >> 20} MiB, "
          f"round exact {ok}", file=sys.stderr, flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
