"""GPU twin of tests/test_cluster_onesided.py: a master process and 4 worker
processes on the box's one MI355X (``--transport onesided``: windows in HBM
mapped through IPC handles, rounds on the gfx950 kernels), thAllreduce =
thReduce = thComplete = 0.75, maxLag 1, one worker's data source sleeping
50 ms per round, 64 rounds: the fast workers' rounds do not wait for it
(its contribution is in few of their chunks), sinks see consistent contributor sets, the
straggler catches up by skipping rounds."""
import pytest

from test_cluster_onesided import check_job, check_late_join

pytestmark = pytest.mark.gpu


def test_cluster_onesided_master_pacing_gpu():
    b, s = check_job("cuda", size=1 << 20, chunk=1 << 16)
    print(f"fast workers' median ms per round: {b:.3f} without, {s:.3f} with the straggler")


def test_cluster_onesided_late_join_gpu():
    """The 4th worker joins after round 5 (master --min-workers 3): the
    members map its window between rounds, it catches up, and from then on
    every block of every round has all 4 contributors (exact thresholds),
    on the card's gfx950 kernels."""
    check_late_join("cuda", size=1 << 20, chunk=1 << 16)
