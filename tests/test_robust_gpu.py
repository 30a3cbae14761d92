"""Robustness of the persistent recurrence inside a training step.

* A hand-off timeout (forced here with a tiny spin limit, dl4ss_debug_set_spin_limit) must
  never reach the weights: the guarded Adam refuses the update on device, the step's loss
  reads NaN, check() raises once and resets the status word, and the next step is normal.
* On the device the plan's grid stays within the co-residency budget (CUs - CUs/16)."""
import numpy as np
import pytest
import torch

from dl4ss_amd import _lib, engine, ops, synth

pytestmark = pytest.mark.gpu


def _batch(dev, B, K, N, seed):
    src, spk, u = synth.SyntheticMixtures(n_samples=N, k=K, seed=seed).batch(B)
    return (torch.from_numpy(src.astype(np.float32)).to(dev),
            torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev),
            torch.from_numpy(spk.astype(np.int32)).to(dev))


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_timed_out_step_never_updates_the_weights(dev, precision):
    B, K, N = 2, 2, 2000
    net = engine.SepNet(cell="lstm", num_layers=2, device=dev, seed=5)
    tr = engine.SepTrainer(net, B, K, N, mode="pit", precision=precision)
    batch = _batch(dev, B, K, N, 5)
    tr.step(*batch)
    tr.check()
    before = (net.flat.clone(), tr.m.clone(), tr.v.clone())
    lib = _lib.lib()
    lib.dl4ss_debug_set_spin_limit(1)  # every poll gives up at once
    try:
        loss = tr.step(*batch)
        torch.cuda.synchronize()
    finally:
        lib.dl4ss_debug_set_spin_limit(0)
    assert int(tr.status.item()) != 0
    assert torch.isnan(loss[0]).item()
    assert torch.equal(net.flat, before[0]) and torch.equal(tr.m, before[1]) and torch.equal(tr.v, before[2])
    with pytest.raises(RuntimeError, match="timed out"):
        tr.check()
    assert int(tr.status.item()) == 0  # reset after reporting
    loss = tr.step(*batch)
    tr.check()
    assert np.isfinite(float(loss[0].item()))
    assert not torch.equal(net.flat, before[0])


def test_device_plan_within_residency_budget(dev):
    cu = torch.cuda.get_device_properties(dev).multi_processor_count
    p = ops.birnn_plan("lstm", 32, 300, "bf16")
    assert p is not None and p["grid"] <= cu - cu // 16
    if cu >= 256:
        assert p["grid"] == 240 and p["BC"] == 4
