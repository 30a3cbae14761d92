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
    assert int(tr.status[0].item()) != 0 and int(tr.status[1].item()) == 1
    assert torch.isnan(loss[0]).item()
    assert torch.equal(net.flat, before[0]) and torch.equal(tr.m, before[1]) and torch.equal(tr.v, before[2])
    n_before = tr.step_count
    with pytest.raises(RuntimeError, match="timed out"):
        tr.check()
    assert tr.status.tolist() == [0, 0]  # reset after reporting
    assert tr.step_count == n_before - 1  # the refused update is not counted (torch Adam's step)
    loss = tr.step(*batch)
    tr.check()
    assert np.isfinite(float(loss[0].item()))
    assert not torch.equal(net.flat, before[0])


def test_peer_timeout_flag_refuses_the_update(dev):
    """Data parallel: a peer rank's timed-out hand-off reaches this rank as a non-zero
    flag behind the flat gradient after the all-reduce (dl4ss_status_flag -> mean).  This
    rank's own status is clean, yet its guarded Adam must refuse the same step (so the replicas
    never drift apart), count the refusal, and check() must raise and roll the step back."""
    B, K, N = 2, 2, 2000
    net = engine.SepNet(cell="lstm", num_layers=2, device=dev, seed=5)
    tr = engine.SepTrainer(net, B, K, N, mode="pit", precision="bf16")
    batch = _batch(dev, B, K, N, 5)
    tr.step(*batch)
    tr.check()
    before = (net.flat.clone(), tr.m.clone(), tr.v.clone())
    n0 = tr.step_count
    tr.spk.copy_(batch[2])
    tr.features(batch[0], batch[1])
    tr.forward()
    loss = tr.loss_and_grad()
    tr.backward()
    # what the all-reduce mean leaves behind when one of two ranks set its flag
    net.dp_flag.fill_(0.5)
    tr.optimizer_step()
    torch.cuda.synchronize()
    assert int(tr.status[0].item()) == 0 and int(tr.status[1].item()) == 1
    assert torch.isnan(loss[0]).item()
    assert torch.equal(net.flat, before[0]) and torch.equal(tr.m, before[1]) and torch.equal(tr.v, before[2])
    with pytest.raises(RuntimeError, match="peer"):
        tr.check()
    assert tr.step_count == n0
    net.dp_flag.zero_()
    loss = tr.step(*batch)
    tr.check()
    assert np.isfinite(float(loss[0].item())) and tr.step_count == n0 + 1


def test_status_flag_kernel(dev):
    st = torch.tensor([0, 0], dtype=torch.int32, device=dev)
    fl = torch.full((1,), 7.0, device=dev)
    _lib.call("dl4ss_status_flag", _lib.ptr(st), _lib.ptr(fl), _lib.stream_ptr())
    assert float(fl.item()) == 0.0
    st[0] = 3
    _lib.call("dl4ss_status_flag", _lib.ptr(st), _lib.ptr(fl), _lib.stream_ptr())
    assert float(fl.item()) == 1.0


def test_device_plan_within_residency_budget(dev):
    cu = torch.cuda.get_device_properties(dev).multi_processor_count
    p = ops.birnn_plan("lstm", 32, 300, "bf16")
    assert p is not None and p["grid"] <= cu - cu // 16
    if cu >= 256:
        assert p["grid"] == 240 and p["BC"] == 4


@pytest.mark.parametrize("cell", ["lstm", "gru"])
def test_write_through_handoff_matches_plain(dev, cell):
    """A recurrence group found on one XCD hands off with plain stores; one that spans XCDs
    writes every granule through (`sc1`).  Forcing the write-through form
    (dl4ss_debug_set_place_force) must give the bitwise-identical bf16 step from the same
    saved state: only the transport differs, never a value.  (B = 4: 120 workgroups in groups
    of 15, the same hand-offs as the B = 32 plan.)"""
    B, K, N = 4, 2, 8000
    lib = _lib.lib()
    net = engine.SepNet(cell=cell, num_layers=2, device=dev, seed=11)
    tr = engine.SepTrainer(net, B, K, N, mode="pit", precision="bf16")
    batch = _batch(dev, B, K, N, 21)
    tr.step(*batch)  # GEMM plans and workspaces exist from here on
    tr.check()
    state = (net.flat.detach().clone(), tr.m.clone(), tr.v.clone(), tr.step_count)
    out = []
    for force in (0, 1):
        net.flat.copy_(state[0]); tr.m.copy_(state[1]); tr.v.copy_(state[2]); tr.step_count = state[3]
        lib.dl4ss_debug_set_place_force(force)
        try:
            loss = tr.step(*batch).clone()
            tr.check()
        finally:
            lib.dl4ss_debug_set_place_force(0)
        out.append((loss, net.grad.detach().clone(), net.flat.detach().clone()))
    (l0, g0, p0), (l1, g1, p1) = out
    assert torch.equal(l0, l1)
    assert torch.equal(g0, g1)
    assert torch.equal(p0, p1)


def test_adam_guarded_keeps_its_one_int_status_contract(dev):
    """the public dl4ss_adam_guarded takes ONE status int (read only); a refusal shows
    only as loss[0] = NaN.  The word after it must stay untouched (an external caller's 1-int
    status would otherwise be written past); the 2-int count lives in dl4ss_adam_guarded_dp."""
    n = 1000
    p = torch.randn(n, device=dev)
    g, m, v = torch.randn(n, device=dev), torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    p0 = p.clone()
    st = torch.tensor([1, 777], dtype=torch.int32, device=dev)
    loss = torch.zeros(1, device=dev)
    _lib.call("dl4ss_adam_guarded", _lib.ptr(p), _lib.ptr(g), _lib.ptr(m), _lib.ptr(v), n, 2e-4, 0.9, 0.999, 1e-8, 1,
              _lib.ptr(st), _lib.ptr(loss), _lib.stream_ptr())
    torch.cuda.synchronize()
    assert st.tolist() == [1, 777] and torch.isnan(loss[0]).item() and torch.equal(p, p0)
    st[0] = 0
    _lib.call("dl4ss_adam_guarded", _lib.ptr(p), _lib.ptr(g), _lib.ptr(m), _lib.ptr(v), n, 2e-4, 0.9, 0.999, 1e-8, 1,
              _lib.ptr(st), _lib.ptr(loss), _lib.stream_ptr())
    torch.cuda.synchronize()
    assert st.tolist() == [0, 777] and not torch.equal(p, p0)
    st = torch.tensor([1, 5], dtype=torch.int32, device=dev)
    ops.adam_(p, g, m, v, 2, status=st, loss=loss)
    torch.cuda.synchronize()
    assert st.tolist() == [1, 6]


def test_dh_split_above_three_fits_the_workspace(dev, monkeypatch):
    """the gemm_gl workspace is sized with the trainer's own dH split
    (DL4SS_DH_SPLIT), so split factors above 3 run instead of raising on the first backward."""
    B, K, N = 4, 2, 4000
    monkeypatch.setenv("DL4SS_DH_SPLIT", "6")
    net = engine.SepNet(cell="lstm", num_layers=2, device=dev, seed=5)
    tr = engine.SepTrainer(net, B, K, N, mode="pit", precision="bf16")
    assert tr.dh_split == 6
    loss = tr.step(*_batch(dev, B, K, N, 6))
    tr.check()
    assert np.isfinite(float(loss[0].item()))


def test_captured_trainer_freed_by_refcount(dev):
    """A trainer that has run eager and graph steps (its CUDAGraph, grouped-GEMM argument arrays,
    workspaces) is freed by reference counting alone once dropped: with the collector off, nothing
    of it can be left for a collection inside a later capture (the round-4 abort;
    tests/test_lifetime_cpu.py pins the same on freshly built trainers)."""
    import gc
    import weakref

    B, K, N = 2, 2, 4000
    batch = _batch(dev, B, K, N, 3)
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        net = engine.SepNet(cell="lstm", num_layers=2, device=dev, seed=3)
        tr = engine.SepTrainer(net, B, K, N, mode="pit", precision="bf16")
        tr.step(*batch)
        tr.step_graph(*batch)
        tr.check()
        refs = [weakref.ref(tr), weakref.ref(tr.graph)] + [weakref.ref(grp) for grp in tr._dw_group]
        del tr
        torch.cuda.synchronize()
        assert all(r() is None for r in refs), [r() is None for r in refs]
        # and the next trainer captures normally
        tr2 = engine.SepTrainer(net, B, K, N, mode="pit", precision="bf16")
        tr2.step(*batch)
        loss = tr2.step_graph(*batch)
        tr2.check()
        assert torch.isfinite(loss[:1]).all()
    finally:
        if was:
            gc.enable()


@pytest.mark.parametrize("cell", ["lstm", "gru"])
def test_recurrence_beside_concurrent_persistent_kernel(dev, cell):
    """A persistent GEMM dispatched on another stream at the same time as the recurrence (the
    side-stream dW_lin; RCCL kernels under data parallelism) interleaves its workgroups into the XCD
    round robin.  The packed kernels form their groups by placement (group_pk: per-XCD slot counters),
    so the roles change but never the arithmetic: forward outputs and BPTT gradients bitwise equal to
    the recurrence run alone, no hand-off timeout."""
    B, T, H = 32, 64, 300
    ng = 4 if cell == "lstm" else 3
    NGH = ng * H
    g = torch.Generator().manual_seed(3)
    G = (torch.randn(B, T, 2, NGH, generator=g) * 0.5).to(dev)
    whh = (torch.randn(2, NGH, H, generator=g) / H ** 0.5).to(dev)
    bhh = (torch.randn(2, NGH, generator=g) * 0.1).to(dev)
    gout = torch.randn(B, T, 2 * H, generator=g).to(dev)
    cellid = 0 if cell == "lstm" else 1
    ws = _lib.query("dl4ss_birnn_workspace_bytes", cellid, B, H)
    # the side GEMM: 16 persistent 256 x 128 workgroups over a long-K problem
    A = ops.to_bf16(torch.randn(8192, 2048, generator=g).to(dev))
    Bm = ops.to_bf16(torch.randn(8192, 512, generator=g).to(dev))
    C = torch.zeros(2048, 512, device=dev)
    side = ops.GroupedGemm([dict(A=A, B=Bm, out=C, transA=True, transB=False, beta=0.0, splitk=1)], dev, grid=16,
                           cfg=2)
    stream = torch.cuda.Stream(device=dev)
    res = []
    for concurrent in (False, True, True):
        o = torch.empty(B, T, 2 * H, device=dev)
        hp = torch.empty_like(o)
        act = torch.empty(B, T, 2, 4 * H, device=dev)
        cs = torch.empty(B, T, 2, H, device=dev)
        dG = torch.zeros(B * T, 2 * NGH, device=dev)
        dGh = torch.zeros_like(dG)
        wsb = torch.zeros((ws + 7) // 8, dtype=torch.int64, device=dev)
        st = torch.zeros(1, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        if concurrent:
            stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(stream):
                side.run()
        _lib.call("dl4ss_birnn_fwd", cellid, 1, B, T, H, _lib.ptr(G), _lib.ptr(whh), _lib.ptr(bhh), _lib.ptr(o),
                  _lib.ptr(hp), _lib.ptr(act), _lib.ptr(cs), _lib.ptr(wsb), ws, _lib.ptr(st), _lib.stream_ptr())
        if concurrent:
            with torch.cuda.stream(stream):
                side.run()
        _lib.call("dl4ss_birnn_bwd", cellid, 1, B, T, H, _lib.ptr(gout), None, _lib.ptr(whh), _lib.ptr(act),
                  _lib.ptr(cs), _lib.ptr(hp), _lib.ptr(dG), _lib.ptr(dGh), _lib.ptr(wsb), ws, _lib.ptr(st),
                  _lib.stream_ptr())
        torch.cuda.synchronize()
        assert int(st.item()) == 0
        res.append((o, dG, dGh))
    for o, dG, dGh in res[1:]:
        assert torch.equal(o, res[0][0]) and torch.equal(dG, res[0][1]) and torch.equal(dGh, res[0][2])
