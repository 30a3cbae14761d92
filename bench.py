"""Benchmark: mixtures/sec of the separation training step on MI355X, 1..8 GPUs of one node.

Workloads (BASELINE.json configs; ``--config``, default C2):

* C2 (default, the headline: configs[1] "2-spk PIT BiLSTM magnitude mask bf16, batch=32"):
  2-speaker synthetic WSJ0-shaped mixtures, 8 kHz, 4 s (N = 32000 -> T = 251, F = 129),
  BiLSTM-4L (H = 300) mask net, Linear(600 -> 129*50) + tanh, embedding + ADDJUST queries,
  PIT MSE + 0.5 sum-to-one loss, backward, DP all-reduce, Adam; bf16 GEMM / recurrent-matvec
  operands with fp32 accumulate, fp32 state, loss, gradients and optimizer -- 32 mixtures per
  GPU per step (weak scaling).
* C4 (configs[3] "3-spk mix at mixed SNR, DP over 8x MI355X with RCCL all-reduce"): 3-speaker
  mixtures with the predata_multiAims_3dB gains, BiGRU-2L without ADDJUST (the selfSS_dB
  model), K = 3 PIT, B = 32 per GPU, one flat RCCL gradient all-reduce per step.
* C5 (configs[4] "recu path, DP over 8x MI355X"): recursive extraction (classifier BiLSTM-3L
  H = 600 + BiGRU-2L mask net, 2 extraction steps, final masks, iSTFT of both estimates),
  B = 1 mixture per replica per step (the reference's batch); replicas only -- no gradients,
  no collective in the step -- and one all-gather of every rank's extracted speaker ids after
  the timed region (the final metric gather).

Inputs (raw sources, gains, speaker ids) are resident in HBM before the timed region; a
training step starts at preprocessing + STFT.

  python bench.py [--gpus N] [--config C2|C4|C5] [--steps K] [--warmup W] [--precision bf16|fp32]
                  [--mode pit|label]

With N > 1 and no WORLD_SIZE in the environment, this process starts the N ranks itself
(``torch.distributed.run`` as a child process, before any GPU call here) and exits with its
code; under torch.distributed.run (the driver's form) WORLD_SIZE must equal --gpus.
``--standin`` replaces the GPU step by a small CPU oracle step over gloo: it exercises only the
launcher, the barrier / max-over-ranks timing and the JSON line (tests/test_bench_launch_cpu.py).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_PEAK = {"fp32": 157.3, "bf16": 2500.0}  # dense TFLOP/s (F32 MFMA / BF16 MFMA)


PMC_TAG = "r06_prof_e"  # tools/prof_round.sh + tools/summarize_prof.py session of this bench command
PMC_FILE = f"profiles/{PMC_TAG}_pmc.json"
MFMA_FILE = f"profiles/{PMC_TAG}_mfma.json"
# the step's GEMM kernels as rocprofv3 names them (MFMA-busy counters are looked up by name): the
# Linear + tanh -> bf16 V (the largest in-step dense contraction) and the input projection (a GEMM
# only on the unfused path: the step forms it inside the recurrence, dl4ss_birnn_fwd_xw)
GEMM_GL_LINEAR = "gemm_gl_kernel<true, true, 2, false, Cfg<128, 2, 64> >"
GEMM_GL_INPROJ = "gemm_gl_kernel<true, true, 0, false, Cfg<128, 2, 64> >"
BW_FILE = "profiles/r03_bw_probe.jsonl"  # tools/bw_probe.hip: plain streaming ceilings on MI355X


def stream_ceiling(kind):
    """Best GB/s of the `kind` stream mix in the committed probe (tools/bw_probe.hip), or None."""
    try:
        with open(os.path.join(ROOT, BW_FILE)) as f:
            rows = [json.loads(l) for l in f if l.strip()]
    except (OSError, ValueError):
        return None
    v = [r["GB/s"] for r in rows if r.get("kernel") == kind]
    return max(v) if v else None


def pmc_mfma_busy(kernel):
    """MFMA-busy fraction of `kernel` (every instantiation, all its dispatches) from the
    committed MFMA / LDS counter pass: SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024
    SIMDs); None if absent."""
    try:
        with open(os.path.join(ROOT, MFMA_FILE)) as f:
            ks = json.load(f)["kernels"]
    except (OSError, KeyError, ValueError):
        return None
    busy = gui = 0.0
    for name, k in ks.items():
        if name == kernel or name.startswith(kernel + "<"):
            busy += k["counters"].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
            gui += k["counters"].get("GRBM_GUI_ACTIVE", 0.0)
    return busy / (gui / 8 * 1024) if gui > 0 else None


def stft_grid_threads(n_sig, T):
    """Launch grid (threads) of dl4ss_stft_fwd: one 256-thread workgroup per 32-frame
    tile (stft.hip)."""
    return n_sig * ((T + 31) // 32) * 256


def stft_grids(B, K, T):
    """The in-step magnitude STFT: ONE launch over the B mixtures + B K sources (the trainer's
    shared signal buffer, SepTrainer._stfts)."""
    return [stft_grid_threads(B + B * K, T)]


def pmc_traffic(kernel, grids):
    """HBM bytes of one measured unit (FETCH_SIZE x2 + WRITE_SIZE, gfx950-corrected) from
    the committed rocprofv3 PMC passes of this same bench command (tools/prof_round.sh +
    tools/summarize_prof.py): the sum over `grids` (launch grid sizes in threads that
    make up the unit) of the average traffic of the launches with that grid; None if
    the summary is absent."""
    path = os.path.join(ROOT, PMC_FILE)
    try:
        with open(path) as f:
            ks = json.load(f)["kernels"]
        # every instantiation of the kernel (templated names: "kernel<...>")
        launches = [l for name, k in ks.items() if name == kernel or name.startswith(kernel + "<")
                    for l in k["launches"]]
    except (OSError, KeyError, ValueError):
        return None
    total = 0.0
    for g in grids:
        v = [l["traffic"] for l in launches if l["grid"] == g]
        if not v:
            return None
        total += sum(v) / len(v)
    return total


CONFIGS = {
    # name: mask net, speakers, per-GPU batch, samples (SURVEY 8 "Configs")
    "C1": dict(kind="cpu", cell="gru", L=2, K=2, adjust=False, B=1, N=40000,
               what="C1: Torch_multi/main_run.py CPU reference path, BiGRU-2L, B=1, dense 101-channel loss"),
    "C2": dict(kind="train", cell="lstm", L=4, K=2, adjust=True, B=32, N=32000,
               what="C2: 2-spk {mode} BiLSTM-4L magnitude mask (EvalVer model)"),
    "C4": dict(kind="train", cell="gru", L=2, K=3, adjust=False, B=32, N=32000,
               what="C4: 3-spk mixed-SNR {mode} BiGRU-2L magnitude mask (selfSS_dB model, 3dB gains)"),
    "C5": dict(kind="recursive", K=2, B=1, N=32000,
               what="C5: recursive extraction replicas (classifier BiLSTM-3L H=600 + BiGRU-2L mask net, "
                    "2 steps, final masks + iSTFT)"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default: the config's)")
    ap.add_argument("--precision", default="bf16", choices=["fp32", "bf16"])
    ap.add_argument("--mode", default="pit", choices=["label", "pit"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true",
                    help="launch every kernel of the step eagerly instead of replaying the captured HIP graph")
    ap.add_argument("--no-stft-standalone", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=6)
    ap.add_argument("--cpu-batch", type=int, default=32)
    ap.add_argument("--dist", action="store_true",
                    help="initialise the RCCL process group even at world size 1 (exercises the DP path)")
    ap.add_argument("--standin", action="store_true",
                    help="CPU stand-in step over gloo (launcher / timing test only; not a measurement)")
    return ap.parse_args(argv)


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """Start n ranks of this script under torch.distributed.run (one process per GPU, RCCL) as
    a CHILD process and return its exit code.  Nothing here has touched the GPU: the parent
    only imported torch, so no initialised HIP runtime is replaced or inherited."""
    import subprocess

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL peer buffers)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    return subprocess.run(cmd, env=env).returncode


def world_from_env(gpus):
    """(world, rank, local rank) of this process; fails loudly when --gpus and the launcher disagree."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: launch N ranks with --gpus N")
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def cpu_threads():
    """Host threads for the CPU baseline: the CPUs this process may run on
    (len(os.sched_getaffinity(0))), capped by the cgroup CPU quota when
    one is set (a container whose affinity lists the whole machine but whose quota is a
    share of it would otherwise oversubscribe its share)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_baseline(args, cfg, with_classifier=False):
    """Reference CPU path (the oracle restatement, torch-CPU fp32 + numpy FFT) on a
    bounded sample of the same workload: cpu_steps steps of the cpu_batch batch.  With
    ``with_classifier`` each step also runs the speaker classifier's forward (BiLSTM-3L,
    H = 600, EvalVer.py:592 / 305-326), which the reference computes and then discards
    (its output is replaced by the ground truth, :598-599): the reference-faithful cost."""
    from oracle import dsp, model as om, recursive as orec
    from dl4ss_amd import synth

    K, N = cfg["K"], cfg["N"]
    cores = cpu_threads()
    torch.set_num_threads(cores)
    torch.manual_seed(1)
    ref = om.SepModel(cell=cfg["cell"], num_layers=cfg["L"], adjust=cfg["adjust"])
    opt = om.make_adam(ref)
    cls = orec.Classifier(hidden=600, num_layers=3) if with_classifier else None
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=1)
    src, spk, u = gen.batch(args.cpu_batch)
    gains = synth.gains_for(u, K)

    def one_step():
        feats, Y = [], []
        for b in range(args.cpu_batch):
            srcs = [dsp.normalise_source(src[b, k], N) for k in range(K)]
            s, m = dsp.mix_sources(srcs, gains[b])
            _ = dsp.stft_tf(m)  # mix_phase (reference computes it, predata_multiAims_dB.py:214)
            feats.append(dsp.magnitude(m))
            Y.append(np.stack([dsp.magnitude(s[k]) for k in range(K)]))
        f = torch.from_numpy(np.array(feats))
        if cls is not None:
            with torch.no_grad():
                cls(f)
        om.train_step(ref, opt, f, f, torch.from_numpy(np.array(Y)), torch.from_numpy(spk), mode=args.mode)

    one_step()  # warm-up
    t0 = time.perf_counter()
    for _ in range(args.cpu_steps):
        one_step()
    dt = time.perf_counter() - t0
    what = "+ classifier BiLSTM-3L H=600 fwd (reference-faithful) " if with_classifier else "(mask path) "
    net = f"{'BiLSTM' if cfg['cell'] == 'lstm' else 'BiGRU'}-{cfg['L']}L"
    return {"value": args.cpu_batch * args.cpu_steps / dt, "unit": "mixtures/s", "cores": cores, "kind": "port",
            "sample": f"{args.cpu_steps} step(s) of the B={args.cpu_batch} batch, oracle torch-CPU fp32 {net} "
                      f"fwd+{args.mode} loss (K={K})+bwd+Adam incl. numpy STFT features {what}on {cores} thread(s)",
            "seconds": dt}


def cpu_reference_c1(args, N, with_classifier=False):
    """BASELINE configs[0]: the CPU reference path of Torch_multi/main_run.py:453-522 on the host
    cores, B = 1, restated on the oracle (torch-CPU fp32 + numpy FFT): features of a synthetic
    2-speaker mixture, MIX_SPEECH BiGRU-2L + Linear + tanh, the DENSE masked embedding of all 101
    labels (main_run.py:307-327, :474), the 'dot' attention over all 101 channels (:478-486), the
    multi-hot mask (:487-489), the 101-channel MSE (:499-506; the sum-to-one term is computed and
    not added, :509-513), backward and Adam.  ``with_classifier``: the discarded
    MIX_SPEECH_classifier forward (:465, BiLSTM H = 300 x NUM_LAYERS = 2, main_run.py:284-305) too."""
    from oracle import dsp, model as om, recursive as orec
    from dl4ss_amd import synth

    K, L = 2, 101
    cores = cpu_threads()
    torch.set_num_threads(cores)
    torch.manual_seed(1)
    ref = om.SepModel(cell="gru", num_layers=2, adjust=False)
    opt = om.make_adam(ref)
    cls = orec.Classifier(hidden=300, num_layers=2) if with_classifier else None
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=1)
    steps = max(1, args.cpu_steps)
    batches = [gen.batch(1) for _ in range(steps + 1)]

    def one_step(src, spk, u):
        gains = synth.gains_for(u, K)
        srcs = [dsp.normalise_source(src[0, k], N) for k in range(K)]
        s, m = dsp.mix_sources(srcs, gains[0])
        _ = dsp.stft_tf(m)  # mix_phase (predata_multiAims.py computes it)
        f = torch.from_numpy(dsp.magnitude(m)[None])
        Y = torch.zeros(1, L, *f.shape[1:])
        for k in range(K):
            Y[0, spk[0, k]] = torch.from_numpy(dsp.magnitude(s[k]))
        topk = torch.zeros(1, L)
        topk[0, torch.from_numpy(spk[0]).long()] = 1.0
        if cls is not None:
            with torch.no_grad():
                cls(f)
        opt.zero_grad()
        V, _ = ref.mix(f)
        q = ref.emb.layer.weight[None] * topk[:, :, None]  # dense embedding x multi-hot
        mask = torch.sigmoid(torch.einsum("btfe,bke->bktf", V, q))
        loss, pred = om.loss_101(mask, topk, f, Y)
        _ = torch.mean((pred.sum(dim=1) - 1.0) ** 2)  # computed, not added (main_run.py:509-513)
        loss.backward()
        opt.step()

    one_step(*batches[0])  # warm-up
    t0 = time.perf_counter()
    for b in batches[1:]:
        one_step(*b)
    dt = time.perf_counter() - t0
    what = "+ discarded classifier BiLSTM-2L H=300 fwd (reference-faithful)" if with_classifier else "(mask path)"
    return {"value": steps / dt, "unit": "mixtures/s", "cores": cores, "kind": "port", "N": N, "T": 1 + N // 128,
            "sample": f"{steps} step(s) at B=1, oracle torch-CPU fp32 BiGRU-2L fwd + 101-channel attention + "
                      f"101-channel MSE + bwd + Adam incl. numpy STFT features {what} on {cores} thread(s)",
            "seconds": dt}


def c1_cpu_lines(args):
    """The four C1 CPU timings SURVEY 8d asks for: N = 40000 (5 s, the reference default) and 32000
    (4 s), each without and with the discarded classifier forward."""
    return {f"N{n}_{tag}": cpu_reference_c1(args, n, with_classifier=wc)
            for n in (40000, 32000) for tag, wc in (("mask_path", False), ("with_classifier", True))}


def c1_main(args):
    """--config C1: BASELINE configs[0], the reference's CPU path (no GPU): one JSON line."""
    lines = c1_cpu_lines(args)
    head = lines["N40000_mask_path"]
    line = {"metric": "mixtures/sec, C1 CPU reference path (Torch_multi/main_run.py, B=1)", "value": head["value"],
            "unit": "mixtures/s", "n_gpus": 0, "steps": args.cpu_steps, "warmup": 1,
            "ms_per_step": 1000.0 / head["value"], "higher_is_better": True, "scaling": None, "vs_baseline": None,
            "dtype": "f32", "data": "synthetic speech-shaped sources, seed 1",
            "config": {"workload": CONFIGS["C1"]["what"], "global_batch": 1, "seq_len": head["T"],
                       "parallelism": "none (host cores)"},
            "cpu_reference_c1": lines}
    print(json.dumps(line), flush=True)


def cpu_baseline_recursive(args, cfg):
    """The oracle's recursive extraction (oracle/recursive.py, GRID.py:383-475) on the host cores,
    one mixture at a time as the reference runs it: numpy STFT features, classifier BiLSTM-3L
    H = 600 and BiGRU-2L mask net twice, final masks (no iSTFT: the GPU line's extra work)."""
    from oracle import dsp, model as om, recursive as orec
    from dl4ss_amd import synth

    N = cfg["N"]
    cores = cpu_threads()
    torch.set_num_threads(cores)
    torch.manual_seed(1)
    mix = om.MixSpeech("gru", 129, 300, 2, 50)
    cls = orec.Classifier(129, 600, 3, 101)
    emb = torch.randn(101, 50)
    gen = synth.SyntheticMixtures(n_samples=N, k=2, seed=5)
    n = max(2, args.cpu_steps)
    src, spk, u = gen.batch(n + 1)
    gains = synth.gains_for(u, 2)

    def one(b):
        _, m = dsp.mix_sources([dsp.normalise_source(src[b, k], N) for k in range(2)], gains[b])
        X = torch.from_numpy(np.asarray(dsp.magnitude(m), np.float32))[None]
        with torch.no_grad():
            orec.recursive_extract(lambda x: mix(x), cls, emb, X)

    one(n)  # warm-up
    t0 = time.perf_counter()
    for b in range(n):
        one(b)
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "mixtures/s", "cores": cores, "kind": "port",
            "sample": f"{n} single-mixture recursive extractions (oracle/recursive.py: classifier BiLSTM-3L H=600 + "
                      f"BiGRU-2L, 2 steps, final masks), torch-CPU fp32 on {cores} thread(s)",
            "seconds": dt}


def standin_main(args, world, rank):
    """--standin: the launcher / timing contract on CPU (gloo).  One 'step' = an oracle training
    step of a tiny BiGRU on this rank's synthetic shard + the flat-gradient all-reduce + Adam."""
    import torch.distributed as dist

    from dl4ss_amd import dp, synth
    from oracle import dsp, model as om

    pg = None
    if world > 1:
        dist.init_process_group("gloo")
        pg = dist.group.WORLD
    torch.set_num_threads(1)
    B, K, N = args.batch or 2, 2, 2000
    torch.manual_seed(0)
    model = om.SepModel(cell="gru", num_layers=1, hidden=32, emb=8)
    params = list(model.parameters())
    flat = torch.cat([p.detach().reshape(-1) for p in params])
    dp.broadcast_params_(flat, pg)
    off = 0
    with torch.no_grad():
        for p in params:
            p.copy_(flat[off:off + p.numel()].view_as(p))
            off += p.numel()
    opt = om.make_adam(model)
    src, spk, u = synth.SyntheticMixtures(n_samples=N, k=K, seed=1, rank=rank).batch(B)
    gains = synth.gains_for(u, K)
    feats, Y = [], []
    for b in range(B):
        s, m = dsp.mix_sources([dsp.normalise_source(src[b, k], N) for k in range(K)], gains[b])
        feats.append(dsp.magnitude(m))
        Y.append(np.stack([dsp.magnitude(s[k]) for k in range(K)]))
    f, Yt, sp = torch.from_numpy(np.array(feats)), torch.from_numpy(np.array(Y)), torch.from_numpy(spk)

    def step():
        opt.zero_grad()
        mask, _, _, _ = model(f, sp)
        loss, _ = om.loss_label_ordered(mask, f, Yt)
        loss.backward()
        g = torch.cat([p.grad.reshape(-1) for p in params])
        work = dp.allreduce_sum_async(g, pg)  # SUM, then the mean's 1 / world (as the trainer's Adam)
        if work is not None:
            work.wait()
            g.mul_(1.0 / dp.world(pg))
        o = 0
        for p in params:
            p.grad.copy_(g[o:o + p.numel()].view_as(p))
            o += p.numel()
        opt.step()
        return float(loss)

    for _ in range(args.warmup):
        step()
    if pg is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    if pg is not None:
        dist.barrier()
    elapsed = dp.max_over_ranks(time.perf_counter() - t0, "cpu", pg)
    # every rank holds the same weights after the synchronous steps
    w = torch.cat([p.detach().reshape(-1) for p in params])
    w_max = dp.max_over_ranks(float(w.sum()), "cpu", pg)
    w_min = -dp.max_over_ranks(-float(w.sum()), "cpu", pg)
    if rank == 0:
        print(json.dumps({"metric": "mixtures/sec (CPU stand-in step; launcher test only, not a measurement)",
                          "value": B * world * args.steps / elapsed, "unit": "mixtures/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
                          "data": "synthetic, CPU stand-in (oracle tiny BiGRU step over gloo)",
                          "config": {"workload": "standin", "global_batch": B * world, "parallelism": f"dp{world}"},
                          "loss": loss, "replicas_in_sync": w_max == w_min}), flush=True)
    if pg is not None:
        dist.destroy_process_group()


def stft_instep_graph(tr, B, K, N, reps=10):
    """The in-step STFT (mixtures and sources, magnitude only: one launch over the trainer's
    shared signal buffer) as the step runs it: captured `reps` times into one HIP graph and
    replayed between two events on the stream the graph runs on, so the per-step time is kernel
    time plus in-graph gaps, not the host launch path of eager re-launches."""

    def pair():
        tr._stfts()

    pair()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            pair()
    g.replay()  # untimed first replay
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (3 * reps)


def stft_standalone(dev, N, T):
    """The north-star STFT roofline measurement: one launch over 4096 signals of N samples,
    complex + magnitude out (>= 2048 signals, ~2.1 GB of traffic per launch), HIP-event average
    of 10 launches on the launch stream (torch's current stream)."""
    from dl4ss_amd import ops

    n_sa = 4096
    xs = torch.randn(n_sa, N, device=dev)
    Xs = torch.empty(n_sa, T, 129, 2, device=dev)
    Ms = torch.empty(n_sa, T, 129, device=dev)
    for _ in range(3):
        ops.stft(xs, out_c=Xs, out_mag=Ms)
    h0, h1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    h0.record()
    for _ in range(10):
        ops.stft(xs, out_c=Xs, out_mag=Ms)
    h1.record()
    torch.cuda.synchronize()
    sa_ms = h0.elapsed_time(h1) / 10
    sa_bytes = n_sa * (4 * N + 12 * T * 129)
    sa_gbs = sa_bytes / (sa_ms * 1e-3) / 1e9
    sa = {"bound": "hbm", "kernel": f"stft_fwd (one launch: {n_sa} signals x N={N}, complex + magnitude; "
                                    "the north-star STFT roofline measurement)",
          "achieved": sa_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": sa_gbs / HBM_PEAK_GBS,
          "traffic": pmc_traffic("stft_fwd_kernel", [stft_grid_threads(n_sa, T)]),
          "traffic_source": PMC_FILE, "launch_ms": sa_ms, "algorithmic_bytes": sa_bytes}
    ceil = stream_ceiling("r1w3")
    if ceil:  # the STFT moves 1 B in : 3 B out; plain streams of that mix peak here
        sa.update({"stream_ceiling": ceil, "frac_of_stream_ceiling": sa_gbs / ceil,
                   "stream_ceiling_source": BW_FILE + " (r1w3: one read : three write streams)"})
    del xs, Xs, Ms
    return sa


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
    torch.cuda.synchronize()


def base_line(args, cfg, world, elapsed, B, T):
    return {
        "metric": "mixtures/sec (8 kHz, 4 s, 2-spk WSJ0-shape) at 1/2/4/8 MI355X",
        "value": B * world * args.steps / elapsed,
        "unit": "mixtures/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.precision == "fp32" else "bf16",
        "data": "synthetic speech-shaped sources (harmonic stack + AM + noise), seed 1+1000*rank, HBM-resident",
        "config": {"workload": cfg["what"].format(mode=args.mode) + f", B={B}/GPU, N={cfg['N']} (T={T},F=129)",
                   "name": args.config, "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world}",
                   "precision": args.precision},
    }


def train_main(args, cfg, dev, world, rank, pg):
    from dl4ss_amd import engine, ops, synth

    B, K, N = args.batch or cfg["B"], cfg["K"], cfg["N"]
    net = engine.SepNet(cell=cfg["cell"], num_layers=cfg["L"], hidden=300, emb=50, num_labels=101,
                        adjust=cfg["adjust"], device=dev, seed=1)
    if world > 1:  # identical initial weights on every rank
        from dl4ss_amd import dp

        dp.broadcast_params_(net.flat, pg)
    tr = engine.SepTrainer(net, B, K, N, mode=args.mode, precision=args.precision, process_group=pg)

    # synthetic input pool, resident in HBM (seed 1 + 1000 * rank)
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=1, rank=rank)
    pool = []
    for _ in range(4):
        src, spk, u = gen.batch(B)
        pool.append((torch.from_numpy(src.astype(np.float32)).to(dev),
                     torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev),
                     torch.from_numpy(spk.astype(np.int32)).to(dev)))

    def timed_step(i):
        raw, gains, spk = pool[i % len(pool)]
        return tr.step_graph(raw, gains, spk) if use_graph else tr.step(raw, gains, spk)

    # HIP graph (default): the step's launches from STFT to the end of backward replay as
    # one graph after an eager warm-up step (workspaces); mixing, the all-reduce and Adam stay
    # eager (engine.SepTrainer.capture)
    use_graph = False
    timed_step(0)
    use_graph = not args.eager
    for i in range(1, max(args.warmup, 1)):
        timed_step(i)
    tr.check()

    barrier(world)
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = timed_step(i)
    barrier(world)
    elapsed = time.perf_counter() - t0
    tr.check()
    if world > 1:
        from dl4ss_amd import dp

        elapsed = dp.max_over_ranks(elapsed, dev, pg)
    loss_v = float(loss[0].item())
    if not np.isfinite(loss_v):
        raise RuntimeError("non-finite loss")

    T = tr.T
    stft_ms = stft_instep_graph(tr, B, K, N)
    stft_bytes = B * (K + 1) * (4 * N + 4 * T * 129)  # mag-only STFT of mixture + K sources
    if getattr(tr, "fast", False):
        stft_bytes += B * T * 129 * 2  # + the mixtures' bf16 magnitudes (the recurrence's input rows, round 5)
    # the MFMA rooflines, each GEMM timed in isolation with the step's own kernel on the step's
    # operands (HIP events around 20 launches on the launch stream):
    #  * Linear + tanh -> bf16 V (M = B*T, N = F*E = 6450, K = 600, bias + tanh fused): the largest
    #    dense contraction inside the step;
    #  * the layer-2 input projection (M = B*T, N = 2 x gates x H, K = 600 + bias) as a GEMM: the
    #    north star's input-projection GEMM, which the step itself forms inside the recurrence kernel
    #    (dl4ss_birnn_fwd_xw), so this is the unfused path's kernel, not an in-step launch.
    bih = net.cat_view("bias_ih", 1)
    ncol = bih.numel()
    FE = 129 * 50

    def time_gemm(fn, reps=20):
        for _ in range(3):
            fn()
        g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        g0.record()
        for _ in range(reps):
            fn()
        g1.record()
        torch.cuda.synchronize()
        return g0.elapsed_time(g1) / reps

    if tr.fast:
        hb = tr.outb[-1][:, :2 * net.H]
        lin_ms = time_gemm(lambda: tr._gemm_fwd(hb, tr.wb_lin[:, :2 * net.H], net.view("mix.Linear.bias"), tr.Vb,
                                                ops.EPI_TANH_BF16))
        lin_kernel = GEMM_GL_LINEAR
        lin_name = f"{lin_kernel} (bf16 operands, in-step Linear {B * T}x{FE}x600 + bias + tanh -> bf16 V)"
        xb, wb = tr.outb[0][:, :2 * net.H], tr.wb_ih[1][:, :2 * net.H]
        inp_ms = time_gemm(lambda: tr._gemm_fwd(xb, wb, bih, tr.G))
        inp_kernel = GEMM_GL_INPROJ
        inp_name = (f"{inp_kernel} (bf16 operands, layer-2 input projection {B * T}x{ncol}x600 + bias as a GEMM; "
                    "the step fuses it into rnn_fwd_pk_kernel)")
    else:
        x, wih = tr.out[0].view(B * T, -1), net.cat_view("weight_ih", 1)
        hL = tr.out[-1].view(B * T, -1)
        lin_ms = time_gemm(lambda: ops.gemm(hL, net.view("mix.Linear.weight"), transB=True,
                                            bias=net.view("mix.Linear.bias"), epilogue=ops.EPI_TANH, out=tr.V,
                                            precision=args.precision))
        lin_kernel = inp_kernel = "gemm_kernel"
        lin_name = f"gemm_kernel (fp32 operands, Linear {B * T}x{FE}x600 + bias + tanh)"
        inp_ms = time_gemm(lambda: ops.gemm(x, wih, transB=True, bias=bih, out=tr.G, precision=args.precision))
        inp_name = f"gemm_kernel (fp32 operands, layer-2 input projection {B * T}x{ncol}x600 + bias)"
    lin_tf = 2.0 * B * T * 600 * FE / (lin_ms * 1e-3) / 1e12
    gemm_tf = 2.0 * B * T * 600 * ncol / (inp_ms * 1e-3) / 1e12
    sa = None if args.no_stft_standalone else stft_standalone(dev, N, T)

    if rank == 0:
        out = base_line(args, cfg, world, elapsed, B, T)
        out["config"].update({"loss": args.mode, "launch": "hip-graph" if use_graph else "eager",
                              "step": "mix+STFT+fwd+loss+bwd+allreduce+Adam"})
        stft_gbs = stft_bytes / (stft_ms * 1e-3) / 1e9
        out.update({
            "loss": loss_v,
            "roofline": sa,
            "roofline_instep": {"bound": "hbm", "kernel": f"stft_fwd in-step (1 launch/step: {B} mixtures + "
                                                         f"{B * K} sources, magnitude; timed as a replayed graph)",
                                "achieved": stft_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": stft_gbs / HBM_PEAK_GBS,
                                "traffic": pmc_traffic("stft_fwd_kernel", stft_grids(B, K, T)),
                                "traffic_source": PMC_FILE, "launch_ms": stft_ms, "algorithmic_bytes": stft_bytes},
            "roofline_mfma": {"bound": "mfma", "kernel": lin_name,
                              "achieved": lin_tf, "peak": MFMA_PEAK[args.precision], "unit": "TFLOP/s",
                              "frac": lin_tf / MFMA_PEAK[args.precision], "launch_ms": lin_ms,
                              "mfma_busy": pmc_mfma_busy(lin_kernel) if args.config == "C2" else None,
                              "mfma_busy_source": MFMA_FILE},
            "roofline_mfma_inproj": {"bound": "mfma", "kernel": inp_name,
                                     "achieved": gemm_tf, "peak": MFMA_PEAK[args.precision], "unit": "TFLOP/s",
                                     "frac": gemm_tf / MFMA_PEAK[args.precision], "launch_ms": inp_ms},
        })
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args, cfg)
            if args.config == "C2":
                out["cpu_baseline_with_classifier"] = cpu_baseline(args, cfg, with_classifier=True)
                # BASELINE configs[0] (the reference's CPU path, B = 1) timed on the same host cores
                out["cpu_reference_c1"] = c1_cpu_lines(args)
        print(json.dumps(out), flush=True)


def recursive_main(args, cfg, dev, world, rank, pg):
    """C5: each rank is an independent replica running the recursive extraction on its own
    synthetic mixtures (B per step, default 1); after the timed region one all-gather brings
    every rank's extracted speaker ids to all ranks (the final metric gather)."""
    from dl4ss_amd import _lib, engine, infer, ops, synth

    B, N = args.batch or cfg["B"], cfg["N"]
    T = ops.n_frames(N)
    net = engine.SepNet(cell="gru", num_layers=2, adjust=False, device=dev, seed=1)
    cnet = infer.ClassifierNet(129, 600, 3, 101, device=dev, seed=2)
    ex = infer.RecursiveExtractor(net, cnet, B, T, precision=args.precision)
    gen = synth.SyntheticMixtures(n_samples=N, k=2, seed=5, rank=rank)
    pool = []
    for _ in range(4):
        src, spk, u = gen.batch(B)
        pool.append((torch.from_numpy(src.astype(np.float32)).to(dev),
                     torch.from_numpy(synth.gains_for(u, 2).astype(np.float32)).to(dev)))
    y = torch.empty(B * 2, 128 * (T - 1), device=dev)
    src_b = torch.empty(B, 2, N, device=dev)
    mix_b = torch.empty(B, N, device=dev)
    stats = torch.empty(32 * B * 2, device=dev)
    Xc = torch.empty(B, T, 129, 2, device=dev)
    Xm = torch.empty(B, T, 129, device=dev)
    pred = torch.empty(B, 2, T, 129, device=dev)
    spk_all = []

    def extract(i):
        raw, gains = pool[i % len(pool)]
        ops.mix_sources(raw, gains, out_src=src_b, out_mix=mix_b, stats_ws=stats)
        ops.stft(mix_b, out_c=Xc, out_mag=Xm)
        out = ex.run(Xm)
        _lib.call("dl4ss_mask_split", _lib.ptr(out["masks"]), _lib.ptr(Xm.unsqueeze(1).expand(B, 2, T, 129)
                                                                         .contiguous()), pred.numel(),
                  _lib.ptr(pred), None, _lib.stream_ptr())
        _lib.call("dl4ss_istft_apply", _lib.ptr(Xc), _lib.ptr(pred), B * 2, 2, T, 0, 0, _lib.ptr(y),
                  _lib.stream_ptr())
        return out

    for i in range(max(args.warmup, 1)):
        extract(i)
    barrier(world)
    t0 = time.perf_counter()
    for i in range(args.steps):
        out = extract(i)
        spk_all.append(out["spk"].clone())
    barrier(world)
    elapsed = time.perf_counter() - t0
    mine = torch.cat(spk_all)  # (steps * B, S) int32 on the device
    if world > 1:
        import torch.distributed as dist

        from dl4ss_amd import dp

        elapsed = dp.max_over_ranks(elapsed, dev, pg)
        gathered = torch.empty(world * mine.shape[0], mine.shape[1], dtype=mine.dtype, device=dev)
        dist.all_gather_into_tensor(gathered, mine, group=pg)
    else:
        gathered = mine
    sa = None if args.no_stft_standalone else stft_standalone(dev, N, T)
    if rank == 0:
        g = gathered.cpu()
        line = base_line(args, cfg, world, elapsed, B, T)
        line["scaling"] = "weak"
        line["config"].update({"replicas": world, "collective": "all_gather of speaker ids after the timed region",
                               "step": "mix+STFT+classifier+2 extraction steps+final masks+iSTFT"})
        line.update({"roofline": sa, "roofline_mfma": None,
                     "gathered_extractions": int(g.shape[0]),
                     "gathered_speakers_found": int((g >= 0).sum()),
                     "speakers_row0": g[0].tolist()})
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline_recursive(args, cfg)
        print(json.dumps(line), flush=True)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # start the ranks before anything touches the GPU; never re-exec this process
        sys.exit(launch_ranks(args.gpus, argv))
    world, rank, local = world_from_env(args.gpus)
    if args.standin:
        return standin_main(args, world, rank)
    cfg = CONFIGS[args.config]
    if cfg["kind"] == "cpu":
        return c1_main(args)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    if world > 1 or args.dist:
        import torch.distributed as dist

        if "RANK" in os.environ:
            dist.init_process_group("nccl", device_id=dev)
        else:  # --dist at world size 1 without a launcher: a private single-rank rendezvous
            dist.init_process_group("nccl", device_id=dev, init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                                    world_size=1)
        pg = dist.group.WORLD
    if cfg["kind"] == "train":
        train_main(args, cfg, dev, world, rank, pg)
    else:
        recursive_main(args, cfg, dev, world, rank, pg)
    if pg is not None:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
