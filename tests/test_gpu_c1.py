"""BASELINE configs[0] end to end on the GPU box: 2-rank loopback allreduce of
1 MiB fp32 (nreduce schedule, gloo transport) whose local reduce steps go
through the drop-in ccl_comp_reduce on host staging buffers; checked with
examples/benchmark's own rule (send = rank, expected (P-1)*P/2)."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fused", [False, True], ids=["chained", "fused_batch"])
@pytest.mark.parametrize("ranks,count", [(2, 262144), (4, 262144), (2, 17 * 2)])
def test_c1_allreduce_through_dropin(ranks, count, fused):
    from tools.c1_allreduce import run
    r = run(ranks, count, 3, "dropin", fused)
    assert r["correct"], r
