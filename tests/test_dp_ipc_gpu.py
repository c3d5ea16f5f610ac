"""Multi-process data-parallel training on the GPU: N ranks
(sharing the box's one GPU) run dp_sgd_step on their own batches, the
gradient buckets meet in the ipc-lane allreduce, and after a few steps
  * every rank holds bit-identical parameters, and
  * they match one process applying the mean of the N ranks' gradients
    (plain autograd + SGD, fp32), to fp32 reduction-order tolerance."""
import os
import socket
import subprocess
import sys
import tempfile

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _reference(n, steps, dev, model_name="mlp"):
    from akka_allreduce_amd.models.mlp import synthetic_batch

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from ddp_ranks import build_model

    torch.manual_seed(0)
    model = build_model(model_name).to(dev)
    for s in range(steps):
        grads = None
        for r in range(n):
            g = torch.Generator(device=dev).manual_seed(100 * s + r)
            x, y = synthetic_batch(64, 256, 10, device=dev, generator=g)
            model.zero_grad(set_to_none=True)
            torch.nn.functional.cross_entropy(model(x), y).backward()
            gr = [p.grad.detach().clone() for p in model.parameters()]
            grads = gr if grads is None else [a + b for a, b in zip(grads, gr)]
        with torch.no_grad():
            for p, g_ in zip(model.parameters(), grads):
                p -= 0.1 * g_ / n
    return torch.cat([p.detach().reshape(-1).float().cpu() for p in model.parameters()])


@pytest.mark.parametrize("n", [2, 3])
def test_dp_sgd_multiprocess_ipc(n):
    steps = 3
    with tempfile.TemporaryDirectory() as out:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               os.path.join(ROOT, "tests", "dp_ranks.py"), "--out-dir", out, "--steps", str(steps)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        res = [torch.load(os.path.join(out, f"rank{i}.pt"), weights_only=True) for i in range(n)]
    diag = _round_diagnosis(res, n, steps)
    for d in res:
        assert d["ipc_error"] == 0 and d["ipc_rounds"] == steps
        assert torch.equal(d["flat"], res[0]["flat"]), diag  # every rank applied the same averaged gradient
    want = _reference(n, steps, torch.device("cuda", 0))
    torch.testing.assert_close(res[0]["flat"], want, rtol=1e-4, atol=1e-5, msg=lambda m: f"{m}\n{diag}")


def _round_diagnosis(res, n, steps) -> str:
    """Per round and rank: does the allreduce output equal the sum of the
    ranks' inputs (which blocks do not)?  Tells a wrong round from a wrong
    update when the final parameters disagree."""
    lines = []
    S = res[0]["rounds_in"][0].numel()
    step = -(-S // n)
    for s in range(steps):
        want = sum(res[i]["rounds_in"][s].double() for i in range(n)).float()
        for i in range(n):
            bad = ((res[i]["rounds_out"][s] - want).abs() > 1e-6 * (1 + want.abs()))
            blocks = [int(bad[b * step:(b + 1) * step].sum()) for b in range(n)]
            lines.append(f"round {s} rank {i}: wrong elements per block {blocks}")
    return "\n".join(lines)


@pytest.mark.parametrize("tune,model", [(False, "mlp"), (True, "mlp"), (True, "deep")])
def test_torch_ddp_hook_multiprocess(tune, model):
    """torch DDP with the comm hook on the ipc data plane, 2 processes: the
    hook's rounds average every bucket across the processes (same result as
    the mean-gradient reference), several bucket sizes -> several allreduce
    engines, all created collectively inside backward, all on one transport
    and one window set, tuned once."""
    n, steps = 2, 3
    with tempfile.TemporaryDirectory() as out:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               os.path.join(ROOT, "tests", "ddp_ranks.py"), "--out-dir", out, "--steps", str(steps),
               "--model", model, "--bucket-mb", "0.3" if model == "deep" else "0.25"]
        if tune:
            cmd.append("--tune")
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        res = [torch.load(os.path.join(out, f"rank{i}.pt"), weights_only=True) for i in range(n)]
    for d in res:
        assert d["ipc_errors"] and all(e == 0 for e in d["ipc_errors"])
        if tune:  # tuned once per hook, the same choice on every rank
            assert all(c and (c.startswith("ipc") or c.startswith("onesided")) for c in d["chosen"]) and d["chosen"] == res[0]["chosen"]
        assert d["buckets"] >= (3 if model == "deep" else 1) and d["rounds"] >= steps
        # every bucket size's engine on ONE transport and ONE set of window memory
        assert d["transports"] == 1 and d["window_sets"] == 1, d
        assert torch.equal(d["flat"], res[0]["flat"])
    want = _reference(n, steps, torch.device("cuda", 0), model)
    torch.testing.assert_close(res[0]["flat"], want, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("bounded", [False, True])
def test_torch_ddp_hook_onesided_multiprocess(bounded):
    """The DDP hook on the one-sided threshold lane (thresholds 1 here, so
    every bucket's mean must equal the mean-gradient reference), 2 processes,
    3 bucket sizes.  ``bounded``: cu_keep=4 sized as on a GPU of its own
    (AKKA_OS_DEDICATED=1 on this 1-GPU box): every round runs on 4 of each 8
    CUs and the hook issues them async (runs_async), overlapping the
    backward on the other CUs."""
    n, steps = 2, 3
    env = dict(os.environ)
    with tempfile.TemporaryDirectory() as out:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               os.path.join(ROOT, "tests", "ddp_ranks.py"), "--out-dir", out, "--steps", str(steps),
               "--model", "deep", "--bucket-mb", "0.3", "--transport", "onesided"]
        if bounded:
            cmd += ["--cu-keep", "4"]
            env["AKKA_OS_DEDICATED"] = "1"
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
        assert r.returncode == 0, r.stderr[-3000:]
        res = [torch.load(os.path.join(out, f"rank{i}.pt"), weights_only=True) for i in range(n)]
    kept = sum(1 for c in range(torch.cuda.get_device_properties(0).multi_processor_count) if c % 8 < 4)
    for d in res:
        assert d["ipc_errors"] and all(e == 0 for e in d["ipc_errors"]), d
        assert d["buckets"] >= 3 and d["rounds"] >= steps
        if bounded:
            assert d["async_rounds"] == d["rounds"] and all(c == kept for c in d["lane_cus"]), d
            assert len(d["cu_streams"]) == 1 and d["cu_streams"][0] != 0, d  # one masked stream per process
        else:
            assert d["async_rounds"] == 0 and all(c == 0 for c in d["lane_cus"]), d
        assert torch.equal(d["flat"], res[0]["flat"])
    want = _reference(n, steps, torch.device("cuda", 0), "deep")
    torch.testing.assert_close(res[0]["flat"], want, rtol=1e-4, atol=1e-5)


def test_torch_ddp_hook_onesided_straggler():
    """The reference's straggler case through torch DDP on the GPU: rank 1
    sleeps 30 ms before each of its bucket rounds; at thresholds 1/2 the
    one-sided rounds of rank 0 complete on what arrived, so rank 0's DDP
    steps (after the first two: engine creation and DDP's bucket rebuild are
    collective) stay far below one straggler delay, with no wait timing out."""
    n, steps, delay_ms = 2, 8, 30
    env = dict(os.environ, AKKA_FAULT_RANK="1", AKKA_FAULT_DELAY_MS=str(delay_ms))
    with tempfile.TemporaryDirectory() as out:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               os.path.join(ROOT, "tests", "ddp_ranks.py"), "--out-dir", out, "--steps", str(steps),
               "--model", "deep", "--bucket-mb", "0.3", "--transport", "onesided", "--th", "0.5"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
        assert r.returncode == 0, r.stderr[-3000:]
        res = [torch.load(os.path.join(out, f"rank{i}.pt"), weights_only=True) for i in range(n)]
    med = [sorted(d["step_s"][2:])[len(d["step_s"][2:]) // 2] for d in res]
    for d in res:
        assert all(e == 0 for e in d["ipc_errors"]), d  # no bounded wait expired
        assert bool(torch.isfinite(d["flat"]).all())
    assert med[1] >= delay_ms / 1e3, med  # the straggler pays its delay per round
    assert med[0] < 0.25 * delay_ms / 1e3, (med, res[0]["step_s"])  # the fast rank never waits for it
