"""Plan selection of the persistent recurrence under a co-residency budget (host-only:
dl4ss_birnn_plan_info with an explicit budget makes no device call).  Every workgroup of
a launch must be resident at once (birnn.hip), so a smaller budget -- a CPX partition, CUs
held by another process -- must widen the batch chunk or refuse the configuration, never
launch a grid that cannot be co-resident."""
import pytest

from dl4ss_amd import ops


@pytest.mark.parametrize("cell,ng", [("lstm", 15), ("gru", 15)])
def test_full_device_plan(cell, ng):
    p = ops.birnn_plan(cell, 32, 300, "bf16", max_wg=240)  # 256 CUs - 1/16
    assert p == {"BC": 4, "NG": ng, "J": 20, "nchunk": 8, "grid": 240}


def test_smaller_budget_widens_the_chunk():
    assert ops.birnn_plan("lstm", 32, 300, "bf16", max_wg=239)["BC"] == 8
    p = ops.birnn_plan("lstm", 32, 300, "bf16", max_wg=120)
    assert p["BC"] == 8 and p["grid"] == 120


def test_budget_too_small_is_refused():
    # a 32-CU partition (budget 30): one chunk of 8 rows at most -> B = 32 cannot run
    assert ops.birnn_plan("lstm", 32, 300, "bf16", max_wg=30) is None
    assert ops.birnn_plan("lstm", 8, 300, "bf16", max_wg=30) == {"BC": 8, "NG": 15, "J": 20, "nchunk": 1, "grid": 30}
    assert ops.birnn_plan("lstm", 1, 300, "bf16", max_wg=29) is None


@pytest.mark.parametrize("B", [1, 2, 3, 5, 16, 31, 32, 33, 64])
def test_grid_never_exceeds_budget(B):
    for budget in (30, 60, 120, 240):
        p = ops.birnn_plan("gru", B, 300, "fp32", max_wg=budget)
        if p is not None:
            assert p["grid"] <= budget and p["BC"] * p["nchunk"] >= B
            # the smallest chunk that fits: one step narrower would not
            if p["BC"] > 1:
                narrower = 2 * ((B + p["BC"] // 2 - 1) // (p["BC"] // 2)) * p["NG"]
                assert narrower > budget


def test_fused_projection_support_is_host_only():
    """dl4ss_birnn_fwd_xw_supported answers from the plan alone (no device call): the packed
    bf16 plan of the nets' H = 300 exists at any batch, input widths up to 2 HMAX = 640; the
    H = 600 classifier has no packed plan."""
    from dl4ss_amd import _lib
    q = lambda *a: _lib.query("dl4ss_birnn_fwd_xw_supported", *a)
    assert q(0, 32, 251, 300, 129) == 1 and q(0, 32, 251, 300, 600) == 1 and q(1, 1, 2, 300, 600) == 1
    assert q(0, 32, 251, 300, 641) == 0
    assert q(0, 32, 251, 600, 600) == 0
    assert q(2, 32, 251, 300, 600) == 0 and q(0, 0, 251, 300, 600) == 0
