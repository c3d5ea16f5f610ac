"""gfx950 kernel numerics vs a plain PyTorch fp32 reference of the same op."""
import pytest
import torch

from akka_allreduce_amd.data import Geometry
from akka_allreduce_amd.ops import chunk_reduce, count_expand

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("impl", ["auto", "vec", "lds", "scalar"])
@pytest.mark.parametrize("nsrc", [1, 2, 3, 7, 8, 9, 16, 17, 23])
@pytest.mark.parametrize("n", [1, 5, 63, 256, 4096 + 3, 1 << 18])
def test_chunk_reduce_fp32(impl, nsrc, n):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(nsrc * 1000 + n)
    srcs = [torch.randn(n, device=dev, generator=g) for _ in range(nsrc)]
    got = chunk_reduce(srcs, impl=impl)
    want = torch.stack(srcs).double().sum(0).float()
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-5 * nsrc)


@pytest.mark.parametrize("impl", ["vec", "lds"])
@pytest.mark.parametrize("nsrc", [1, 2, 4, 8, 16])
@pytest.mark.parametrize("n", [7, 1024, 100_003])
def test_chunk_reduce_bf16(impl, nsrc, n):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(nsrc + n)
    srcs = [torch.randn(n, device=dev, generator=g).bfloat16() for _ in range(nsrc)]
    got = chunk_reduce(srcs, impl=impl)
    want = torch.stack([s.float() for s in srcs]).sum(0).bfloat16()  # fp32 accumulate, one rounding
    assert torch.equal(got, want)


def test_chunk_reduce_unaligned_views():
    dev = torch.device("cuda")
    base = [torch.randn(10_001, device=dev) for _ in range(3)]
    srcs = [b[1:] for b in base]  # 4-byte offset: not 16-B aligned -> scalar path
    got = chunk_reduce(srcs)
    torch.testing.assert_close(got, torch.stack(srcs).sum(0))


def test_chunk_reduce_large_exact():
    dev = torch.device("cuda")
    n = (64 << 20) // 4
    srcs = [torch.full((n,), float(i + 1), device=dev) for i in range(8)]
    for impl in ("vec", "lds"):
        got = chunk_reduce(srcs, impl=impl)
        assert bool((got == 36.0).all()), impl


@pytest.mark.parametrize("S,N,C", [(3, 2, 2), (778, 4, 3), (16, 3, 2), (5, 4, 1), (1 << 20, 8, 4096), (1000, 7, 64)])
def test_count_expand(S, N, C):
    g = Geometry(S, N, C)
    per = torch.randint(0, 9, (N, g.kmax), dtype=torch.int32)
    want = g.expand_counts(per)
    got = count_expand(per.cuda(), g).cpu()
    assert torch.equal(got, want)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("off", [1, 2, 3, 5, 7])
@pytest.mark.parametrize("nsrc", [1, 3, 8])
def test_chunk_reduce_common_misalignment(dtype, off, nsrc):
    """All pointers at the same offset mod 16 B (the data plane's layout):
    the launcher peels a scalar head and runs the vector body; results must
    match the fp32 reference exactly for small-integer data."""
    n = 100_003
    base = [torch.randint(-8, 9, (n + 16,), device="cuda").to(dtype) for _ in range(nsrc)]
    srcs = [b[off:off + n] for b in base]
    out_base = torch.empty(n + 16, device="cuda", dtype=dtype)
    out = out_base[off:off + n]
    chunk_reduce(srcs, out=out)
    want = torch.stack([x.float() for x in srcs]).sum(0).to(dtype)
    assert torch.equal(out, want)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("S,N,C", [(1000, 4, 64), (100_003, 3, 777), (5, 4, 1), (1 << 20, 8, 1 << 14), (77, 2, 100)])
def test_count_mean_matches_torch(dtype, S, N, C):
    """Fused AllReduceOutput.mean (count_mean kernel) == torch.where(c>0, x/c, 0)
    with per-element counts expanded from the per-chunk table (incl. zeros)."""
    from akka_allreduce_amd.data import AllReduceOutput

    g = Geometry(S, N, C)
    x = torch.randn(S, device="cuda").to(dtype)
    pc = torch.randint(0, N + 1, (N, g.kmax), device="cuda", dtype=torch.int32)
    o = AllReduceOutput(x, counts_per_chunk=pc, geometry=g)
    got = o.mean()
    c = g.expand_counts(pc.cpu()).cuda().to(dtype)
    want = torch.where(c > 0, x / c.clamp(min=1), torch.zeros_like(x))
    assert torch.equal(got, want)
    buf = torch.empty_like(x)
    assert o.mean(out=buf) is buf and torch.equal(buf, want)
