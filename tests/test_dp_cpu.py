"""Multi-rank data parallelism on CPU (gloo, world_size 2): the same host calls the
GPU path makes over RCCL (dl4ss_amd.dp), checked against a single-process run of
the oracle step on the global batch.

Rank r generates its own synthetic shard (seed 1 + 1000 r, as bench.py), computes
the oracle loss / gradients on it, all-reduces the flat gradient with the trainer's own
helpers (dp.allreduce_sum_async / dp.allreduce_buckets_: a SUM, the 1 / world of the mean
applied as Adam's gradient scale, as dl4ss_adam_guarded_dp_scaled does) and takes an Adam step; the result must equal the single-process step on the concatenated
global batch (the reference's objective: MSE means over the whole batch)."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dl4ss_amd import dp, synth
from oracle import dsp, model as om

N = 2000
K = 2
B_PER_RANK = 2


def _features(src, gains):
    feats, Y = [], []
    for b in range(src.shape[0]):
        srcs = [dsp.normalise_source(src[b, k].astype(np.float32), N) for k in range(K)]
        s, m = dsp.mix_sources(srcs, gains[b])
        feats.append(np.abs(dsp.stft_tf(m)))
        Y.append(np.stack([np.abs(dsp.stft_tf(s[k])) for k in range(K)]))
    return torch.from_numpy(np.array(feats, np.float32)), torch.from_numpy(np.array(Y, np.float32))


def _shard(rank):
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=1, rank=rank)
    src, spk, u = gen.batch(B_PER_RANK)
    f, Y = _features(src, synth.gains_for(u, K))
    return f, Y, torch.from_numpy(spk)


def _model():
    torch.manual_seed(0)
    return om.SepModel(cell="gru", num_layers=1, hidden=32, emb=8)


def _flat_grads(model):
    return torch.cat([p.grad.reshape(-1) for p in model.parameters()])


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    model = _model()
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    if rank == 1:
        flat.add_(1.0)  # diverged init: broadcast must restore rank 0's weights
    dp.broadcast_params_(flat)
    off = 0
    with torch.no_grad():
        for p in model.parameters():
            p.copy_(flat[off:off + p.numel()].view_as(p))
            off += p.numel()
    f, Y, spk = _shard(rank)
    opt = om.make_adam(model)
    opt.zero_grad()
    mask, _, _, _ = model(f, spk)
    loss, _ = om.loss_label_ordered(mask, f, Y)
    loss.backward()
    g = _flat_grads(model)
    work = dp.allreduce_sum_async(g)  # SepTrainer.allreduce
    work.wait()
    g = g * (1.0 / dp.world())  # the guarded Adam's gscale = 1 / world (engine.SepTrainer.optimizer_step)
    off = 0
    for p in model.parameters():
        p.grad.copy_(g[off:off + p.numel()].view_as(p))
        off += p.numel()
    opt.step()
    tmax = dp.max_over_ranks(float(rank + 1), "cpu")
    out[rank] = (g.clone(), torch.cat([p.detach().reshape(-1) for p in model.parameters()]), tmax)
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_dp_two_ranks_equals_global_batch():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    # single-process reference on the global batch (rank shards concatenated)
    shards = [_shard(r) for r in range(world)]
    f = torch.cat([s[0] for s in shards])
    Y = torch.cat([s[1] for s in shards])
    spk = torch.cat([s[2] for s in shards])
    model = _model()
    opt = om.make_adam(model)
    opt.zero_grad()
    mask, _, _, _ = model(f, spk)
    loss, _ = om.loss_label_ordered(mask, f, Y)
    loss.backward()
    g_ref = _flat_grads(model)
    opt.step()
    p_ref = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    for r in range(world):
        g, p, tmax = out[r]
        assert torch.allclose(g, g_ref, rtol=1e-4, atol=1e-7), (g - g_ref).abs().max()
        # Adam's first step lr g / (|g| + eps) is steep near |g| ~ eps (d/dg = lr eps / (|g| + eps)^2): the
        # summation-order difference of the two-rank gradient moves such weights by up to that slope x the
        # measured gradient difference (2.4e-9 gradients moved 3.6e-7 on one run)
        err = float((g - g_ref).abs().max())
        lr, eps = 2e-4, 1e-8
        tol = 1e-7 + 1e-5 * p_ref.abs() + 4 * lr * err * eps / (g_ref.abs() + eps) ** 2
        assert bool(((p - p_ref).abs() <= tol).all()), (p - p_ref).abs().max()
        assert tmax == 2.0
    # the two ranks' synthetic shards are different utterances
    assert not torch.equal(shards[0][0], shards[1][0])


def _flag_worker(rank, world, port, out):
    """The hand-off status flag rides behind the flat gradient through the SUM all-reduce
    (engine.SepNet.grad_ext / SepTrainer.allreduce): one rank's timeout reaches every rank."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = []
    for bad in (None, 1, 0):  # no rank timed out / rank 1 / rank 0
        grad_ext = torch.zeros(8 + 4)
        grad_ext[:8] = float(rank + 1)
        grad_ext[8] = 1.0 if rank == bad else 0.0  # dl4ss_status_flag
        dp.allreduce_sum_async(grad_ext).wait()
        res.append((float(grad_ext[0]) / world, float(grad_ext[8])))
    out[rank] = res
    dist.destroy_process_group()


def test_dp_status_flag_reaches_every_rank():
    world = 3
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_flag_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        (g0, f0), (g1, f1), (g2, f2) = out[r]
        assert g0 == g1 == g2 == 2.0  # the gradient (its mean) is unaffected by the flag slot
        assert f0 == 0.0  # clean step: every rank's guarded Adam applies it
        assert f1 > 0.0 and f2 > 0.0  # a timeout on any one rank: every rank refuses the step


def _bucket_worker(rank, world, port, out):
    """The bucketed all-reduce of the trainer's extended gradient [flag | layers | Linear, emb, adj]
    (SepTrainer.allreduce_early / allreduce_late: two async SUMs split at SepNet.bucket_split) against
    one flat SUM (SepTrainer.allreduce), on the layout of the C2 net."""
    from dl4ss_amd import engine

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    net = engine.SepNet(cell="lstm", num_layers=4, device="cpu")
    g = torch.Generator().manual_seed(100 + rank)
    ext = torch.randn(net.grad_ext.numel(), generator=g) * (1 + rank)
    ext[0] = 1.0 if rank == 1 else 0.0  # rank 1's hand-off timed out (dl4ss_status_flag)
    flat = ext.clone()
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    buck = dp.allreduce_buckets_(ext.clone(), net.bucket_split())
    # three buckets (round 6): layers < L // 2 with the flag, layers >= L // 2, Linear / emb / ADDJUST
    buck3 = dp.allreduce_buckets_(ext.clone(), [net.bucket_mid(net.L // 2), net.bucket_split()])
    out[rank] = (flat, buck, buck3)
    dist.destroy_process_group()


def test_dp_bucketed_allreduce_equals_flat():
    from dl4ss_amd import engine

    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_bucket_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    net = engine.SepNet(cell="lstm", num_layers=4, device="cpu")
    split = net.bucket_split()
    # the buckets are the contiguous ranges the backward completes at different times
    early = {n for n, (off, _) in net.offsets.items() if off + 4 >= split}
    assert early == {"mix.Linear.weight", "mix.Linear.bias", "emb.layer.weight", "adj.layer.weight"}
    assert net.dp_flag.data_ptr() == net.grad_ext.data_ptr()  # the flag travels with the late bucket
    mid = net.bucket_mid(net.L // 2)  # the three-bucket step's middle bucket: exactly layers 2 and 3 of C2
    middle = {n for n, (off, _) in net.offsets.items() if mid <= off + 4 < split}
    assert middle == {f"mix.layer.{kind}_l{l}{rev}" for kind in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")
                      for l in (2, 3) for rev in ("", "_reverse")}
    for r in range(world):
        flat, buck, buck3 = out[r]
        assert torch.equal(flat, buck)  # bitwise: the same elementwise sums
        assert torch.equal(flat, buck3)
        assert torch.equal(flat, out[0][0])  # every rank holds the same sums
        assert flat[0] == 1.0  # one rank's timeout reaches every rank through the late bucket
    # (Adam's 1 / world on the SUM, dl4ss_adam_guarded_dp_scaled, runs on the GPU:
    # tests/test_step_gpu.py::test_dp_scaled_adam_on_summed_half_batches_equals_full_batch_step)
