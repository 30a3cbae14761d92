"""The data-parallel path on the GPU at world size 1 over RCCL: an ``nccl``
process group with a private TCP rendezvous (as ``bench.py --dist``), and SepTrainer's graph
step with ``process_group=pg`` -- status flag in front of the flat gradient -> RCCL SUM all-reduce of
``grad_ext`` (three buckets, two, or flat) -> ``dl4ss_adam_guarded_dp_scaled`` (x 1 / world) -- beside the
240-workgroup persistent recurrence and the side-stream dW_lin.

* At world size 1 the all-reduce is an identity, so the pg step must be BITWISE the pg=None step:
  losses, gradients, parameters, Adam moments and the status word, over several steps, for C2
  (BiLSTM-4L, K = 2) and C4 (BiGRU-2L, K = 3) at the benched size (B = 32, N = 32000).
* A forced hand-off timeout (dl4ss_debug_set_spin_limit) travels through the real all-reduce as
  the status flag and the guarded Adam refuses the update (the DP refusal path, not a faked flag).
"""
import gc
import socket

import numpy as np
import pytest
import torch

from dl4ss_amd import _lib, engine, synth

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def pg(dev):
    import torch.distributed as dist

    if dist.is_initialized():
        pytest.skip("a process group already exists in this process")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev, init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1)
    yield dist.group.WORLD
    dist.destroy_process_group()


CFGS = {"C2": dict(cell="lstm", L=4, K=2, adjust=True), "C4": dict(cell="gru", L=2, K=3, adjust=False)}


def _pool(dev, B, K, N, n=3):
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=1)
    out = []
    for _ in range(n):
        src, spk, u = gen.batch(B)
        out.append((torch.from_numpy(src.astype(np.float32)).to(dev),
                    torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev),
                    torch.from_numpy(spk.astype(np.int32)).to(dev)))
    return out


def _trainer(dev, cfg, B, K, N, pg):
    net = engine.SepNet(cell=cfg["cell"], num_layers=cfg["L"], hidden=300, emb=50, num_labels=101,
                        adjust=cfg["adjust"], device=dev, seed=1)
    return engine.SepTrainer(net, B, K, N, mode="pit", precision="bf16", process_group=pg)


@pytest.mark.parametrize("name,buckets", [("C2", "3"), ("C4", "3"), ("C2", "2"), ("C2", "0")])
def test_rccl_world1_graph_step_bitwise_equal_to_single_gpu(dev, pg, name, buckets, monkeypatch):
    """buckets "3" (round 6, not the default): the early bucket (Linear, embedding, ADDJUST) all-reduced after
    the BPTT chain beside the upper layers' weight-gradient launch, the upper layers' bucket beside the
    lower layers' launch, the lower layers + status flag last, three graph replays; "2" (the default, round 5): the
    early bucket, then every layer + the flag after one weight-gradient launch, two replays; "0": one
    flat all-reduce after one replay.  All SUM, with the 1 / world inside Adam."""
    monkeypatch.setenv("DL4SS_DP_BUCKETS", buckets)
    cfg = CFGS[name]
    B, K, N = 32, cfg["K"], 32000
    pool = _pool(dev, B, K, N)
    runs = {}
    for tag, group in (("single", None), ("rccl", pg)):
        tr = _trainer(dev, cfg, B, K, N, group)
        assert tr.buckets == (group is not None and buckets != "0")
        assert (tr.dp_layer is not None) == (group is not None and buckets == "3")
        tr.step(*pool[0])  # eager warm-up before the capture
        losses = [float(tr.step_graph(*b)[0].item()) for b in pool]
        tr.check()
        torch.cuda.synchronize()
        runs[tag] = dict(loss=losses, grad=tr.net.grad_ext.clone(), flat=tr.net.flat.clone(), m=tr.m.clone(),
                         v=tr.v.clone(), status=tr.status.tolist(), steps=tr.step_count)
        del tr
        gc.collect()
        torch.cuda.empty_cache()
    a, b = runs["single"], runs["rccl"]
    assert all(np.isfinite(a["loss"])) and a["loss"] == b["loss"]
    assert a["steps"] == b["steps"] == len(pool) + 1 and a["status"] == b["status"] == [0, 0]
    for k in ("grad", "flat", "m", "v"):
        assert torch.equal(a[k], b[k]), k


def test_rccl_world1_forced_timeout_refused_through_allreduce(dev, pg):
    """The timed-out step's status flag is written in front of the flat gradient, goes through the
    RCCL all-reduce, and the guarded DP Adam refuses the update: weights and moments untouched,
    loss NaN, check() raises and rolls the step count back, the next step is normal."""
    B, K, N = 4, 2, 8000
    cfg = dict(cell="lstm", L=2, adjust=True)
    pool = _pool(dev, B, K, N, n=1)
    tr = _trainer(dev, cfg, B, K, N, pg)
    tr.step(*pool[0])
    tr.check()
    before = (tr.net.flat.clone(), tr.m.clone(), tr.v.clone())
    n0 = tr.step_count
    lib = _lib.lib()
    lib.dl4ss_debug_set_spin_limit(1)  # every poll gives up at once
    try:
        loss = tr.step(*pool[0])  # eager: the spin limit is a launch argument
        torch.cuda.synchronize()
    finally:
        lib.dl4ss_debug_set_spin_limit(0)
    assert int(tr.status[0].item()) != 0 and int(tr.status[1].item()) == 1
    assert float(tr.net.dp_flag[0].item()) == 1.0  # the flag as the all-reduce left it
    assert torch.isnan(loss[0]).item()
    assert torch.equal(tr.net.flat, before[0]) and torch.equal(tr.m, before[1]) and torch.equal(tr.v, before[2])
    with pytest.raises(RuntimeError, match="timed out"):
        tr.check()
    assert tr.step_count == n0 and tr.status.tolist() == [0, 0]
    loss = tr.step(*pool[0])
    tr.check()
    assert np.isfinite(float(loss[0].item())) and tr.step_count == n0 + 1
