"""Benchmark: mixtures/sec of the full separation training step on MI355X.

Workload (BASELINE.json configs[1] "2-spk PIT BiLSTM magnitude mask bf16, batch=32",
SURVEY section 8d C2): 2-speaker synthetic WSJ0-shaped mixtures, 8 kHz, 4 s
(N = 32000 -> T = 251, F = 129), BiLSTM-4L (H = 300) mask net, Linear(600 -> 129*50)
+ tanh, embedding + ADDJUST queries, PIT MSE + 0.5 sum-to-one loss, backward,
(DP all-reduce), Adam; bf16 GEMM / recurrent-matvec operands with fp32 accumulate,
fp32 state, loss, gradients and optimizer --
32 mixtures per GPU per step (weak scaling).  Inputs (raw sources, gains,
speaker ids) are resident in HBM before the timed region; the step starts at
preprocessing + STFT.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--precision bf16|fp32] [--mode pit|label]

N > 1 is launched by torch.distributed.run (one rank per GPU, RCCL).
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


PMC_TAG = "r02_prof_e"  # tools/prof_round.sh + tools/summarize_prof.py session of this bench command
PMC_FILE = f"profiles/{PMC_TAG}_pmc.json"
MFMA_FILE = f"profiles/{PMC_TAG}_mfma.json"
# the in-step input-projection kernel as rocprofv3 names it (its MFMA-busy counter is looked up by it)
GEMM_GL_INPROJ = "gemm_gl_kernel<true, true, 0, false, Cfg<128, 2> >"
BW_FILE = "profiles/r02_bw_probe.jsonl"  # tools/bw_probe.hip: plain 16-B streaming ceilings on MI355X


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
    return [stft_grid_threads(B, T), stft_grid_threads(B * K, T)]


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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
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
    return ap.parse_args()


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


def cpu_baseline(args, N, K, with_classifier=False):
    """Reference CPU path (the oracle restatement, torch-CPU fp32 + numpy FFT) on a
    bounded sample of the same workload: cpu_steps steps of the B = 32 batch.  With
    ``with_classifier`` each step also runs the speaker classifier's forward (BiLSTM-3L,
    H = 600, EvalVer.py:592 / 305-326), which the reference computes and then discards
    (its output is replaced by the ground truth, :598-599): the reference-faithful cost."""
    from oracle import dsp, model as om, recursive as orec
    from dl4ss_amd import synth

    cores = cpu_threads()
    torch.set_num_threads(cores)
    torch.manual_seed(1)
    ref = om.SepModel(cell="lstm", num_layers=4)
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
    return {"value": args.cpu_batch * args.cpu_steps / dt, "unit": "mixtures/s", "cores": cores, "kind": "port",
            "sample": f"{args.cpu_steps} step(s) of the B={args.cpu_batch} batch, oracle torch-CPU fp32 BiLSTM-4L "
                      f"fwd+{args.mode} loss+bwd+Adam incl. numpy STFT features {what}on {cores} thread(s)",
            "seconds": dt}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    if world > 1 or args.dist:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)
        pg = dist.group.WORLD

    from dl4ss_amd import engine, ops, synth

    B, K, N = args.batch, 2, 32000
    net = engine.SepNet(cell="lstm", num_layers=4, hidden=300, emb=50, num_labels=101, device=dev, seed=1)
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

    # per-phase HIP events on the stream the kernels run on (torch's current stream)
    ev = {"stft": []}

    def timed_step(i, record):
        raw, gains, spk = pool[i % len(pool)]
        if use_graph:
            return tr.step_graph(raw, gains, spk)
        if not record:
            return tr.step(raw, gains, spk)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        tr.spk.copy_(spk)
        ops.mix_sources(raw, gains, out_src=tr.src, out_mix=tr.mix, stats_ws=tr.stats)
        e0.record()  # the two STFT launches (mixtures, then sources) of engine.SepTrainer.features
        ops.stft(tr.mix, complex_out=False, mag_out=True, out_mag=tr.mag_mix)
        ops.stft(tr.src.view(B * K, N), complex_out=False, mag_out=True, out_mag=tr.mag_src.view(B * K, tr.T, tr.F))
        e1.record()
        ev["stft"].append((e0, e1))
        tr.forward()
        loss = tr.loss_and_grad()
        tr.backward()
        tr.allreduce()
        tr.optimizer_step()
        return loss

    # HIP graph (default): the step's launches from STFT to the end of backward replay as
    # one graph after an eager warm-up step (GEMM plans, workspaces); mixing, the all-reduce
    # and Adam stay eager (engine.SepTrainer.capture)
    use_graph = False
    timed_step(0, False)
    use_graph = not args.eager
    for i in range(1, max(args.warmup, 1)):
        timed_step(i, False)
    tr.check()

    def barrier():
        if world > 1:
            import torch.distributed as dist

            dist.barrier()
        torch.cuda.synchronize()

    barrier()
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    s0.record()
    for i in range(args.steps):
        loss = timed_step(i, True)
    s1.record()
    barrier()
    elapsed = time.perf_counter() - t0
    tr.check()
    if world > 1:
        from dl4ss_amd import dp

        elapsed = dp.max_over_ranks(elapsed, dev, pg)
    loss_v = float(loss[0].item())
    if not np.isfinite(loss_v):
        raise RuntimeError("non-finite loss")

    if use_graph:  # the in-step STFT launches, timed eagerly on the step's buffers (one untimed pair first)
        ops.stft(tr.mix, complex_out=False, mag_out=True, out_mag=tr.mag_mix)
        ops.stft(tr.src.view(B * K, N), complex_out=False, mag_out=True, out_mag=tr.mag_src.view(B * K, tr.T, tr.F))
        for _ in range(args.steps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.stft(tr.mix, complex_out=False, mag_out=True, out_mag=tr.mag_mix)
            ops.stft(tr.src.view(B * K, N), complex_out=False, mag_out=True, out_mag=tr.mag_src.view(B * K, tr.T, tr.F))
            e1.record()
            ev["stft"].append((e0, e1))
        torch.cuda.synchronize()

    # ---- roofline of the two north-star kernels (STFT in-step events; input GEMM isolated), same stream
    T, F = tr.T, tr.F
    stft_ms = float(np.mean([a.elapsed_time(b) for a, b in ev["stft"]]))
    stft_bytes = B * (K + 1) * (4 * N + 4 * T * F)  # mag-only STFT of mixture + K sources
    # input-projection GEMM of BiLSTM layer 2 (M = B*T, N = 2400, K = 600, bias fused), timed in
    # isolation with the step's own kernel and operands: in bf16 mode gemm_gl.hip on the bf16 h
    # the layer-1 recurrence wrote and the bf16 W_ih copy (the in-step launch), else gemm.hip fp32
    bih = net.cat_view("bias_ih", 1)
    if tr.fast:
        xb, wb = tr.outb[0][:, :2 * net.H], tr.wb_ih[1][:, :2 * net.H]
        run_gemm = lambda: tr._gemm_fwd(xb, wb, bih, tr.G)  # noqa: E731
        gemm_kernel = GEMM_GL_INPROJ if tr.gemm_path == "gl" else "gemm_bb_kernel"
        gemm_name = f"{gemm_kernel} (bf16 operands, in-step BiLSTM layer-2 input projection 8032x2400x600 + bias)"
    else:
        x, wih = tr.out[0].view(B * T, -1), net.cat_view("weight_ih", 1)
        run_gemm = lambda: ops.gemm(x, wih, transB=True, bias=bih, out=tr.G, precision=args.precision)  # noqa: E731
        gemm_kernel = "gemm_kernel"
        gemm_name = "gemm_kernel (fp32 operands, BiLSTM layer-2 input projection 8032x2400x600 + bias)"
    for _ in range(3):
        run_gemm()
    g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g0.record()
    for _ in range(20):
        run_gemm()
    g1.record()
    torch.cuda.synchronize()
    gemm_ms = g0.elapsed_time(g1) / 20
    gemm_flops = 2.0 * B * T * 600 * 2400
    # standalone STFT at the north-star measurement size (>= 2048 signals, ~1 GB of
    # traffic per launch, complex + magnitude outputs): the >= 50 % HBM target.  4096
    # signals (2.1 GB per launch) amortise the launch's ramp-up and drain better
    sa = None
    if not args.no_stft_standalone:
        n_sa = 4096
        xs = torch.randn(n_sa, N, device=dev)
        Xs = torch.empty(n_sa, T, F, 2, device=dev)
        Ms = torch.empty(n_sa, T, F, device=dev)
        for _ in range(3):
            ops.stft(xs, out_c=Xs, out_mag=Ms)
        h0, h1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        h0.record()
        for _ in range(10):
            ops.stft(xs, out_c=Xs, out_mag=Ms)
        h1.record()
        torch.cuda.synchronize()
        sa_ms = h0.elapsed_time(h1) / 10
        sa_bytes = n_sa * (4 * N + 12 * T * F)
        sa_gbs = sa_bytes / (sa_ms * 1e-3) / 1e9
        sa = {"bound": "hbm", "kernel": f"stft_fwd (one launch: {n_sa} signals x N=32000, complex + magnitude; "
                                        "the north-star STFT roofline measurement)",
              "achieved": sa_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": sa_gbs / HBM_PEAK_GBS,
              "traffic": pmc_traffic("stft_fwd_kernel", [stft_grid_threads(n_sa, T)]),
              "traffic_source": PMC_FILE, "launch_ms": sa_ms, "algorithmic_bytes": sa_bytes}
        ceil = stream_ceiling("r1w3")
        if ceil:  # the STFT moves 1 B in : 3 B out; plain streams of that mix peak here
            sa.update({"stream_ceiling": ceil, "frac_of_stream_ceiling": sa_gbs / ceil,
                       "stream_ceiling_source": BW_FILE + " (r1w3: one 16-B read : three 16-B write streams)"})
        del xs, Xs, Ms

    if rank == 0:
        value = B * world * args.steps / elapsed
        stft_gbs = stft_bytes / (stft_ms * 1e-3) / 1e9
        gemm_tf = gemm_flops / (gemm_ms * 1e-3) / 1e12
        out = {
            "metric": "mixtures/sec (8 kHz, 4 s, 2-spk WSJ0-shape) at 1/2/4/8 MI355X",
            "value": value,
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
            "config": {"workload": f"C2: 2-spk {args.mode} BiLSTM-4L magnitude mask, B=32/GPU, N=32000 (T=251,F=129),"
                                   " full step: mix+STFT+fwd+loss+bwd+allreduce+Adam",
                       "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world}",
                       "precision": args.precision, "loss": args.mode,
                       "launch": "hip-graph" if use_graph else "eager"},
            "loss": loss_v,
            "roofline": sa,
            "roofline_instep": {"bound": "hbm", "kernel": "stft_fwd in-step (2 launches/step: 32 mixtures + 64 "
                                                         "sources, magnitude)",
                                "achieved": stft_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": stft_gbs / HBM_PEAK_GBS,
                                "traffic": pmc_traffic("stft_fwd_kernel", stft_grids(B, K, T)),
                                "traffic_source": PMC_FILE, "launch_ms": stft_ms, "algorithmic_bytes": stft_bytes},
            "roofline_mfma": {"bound": "mfma", "kernel": gemm_name,
                              "achieved": gemm_tf, "peak": MFMA_PEAK[args.precision], "unit": "TFLOP/s",
                              "frac": gemm_tf / MFMA_PEAK[args.precision], "launch_ms": gemm_ms,
                              "mfma_busy": pmc_mfma_busy(gemm_kernel), "mfma_busy_source": MFMA_FILE},
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args, N, K)
            out["cpu_baseline_with_classifier"] = cpu_baseline(args, N, K, with_classifier=True)
        print(json.dumps(out), flush=True)
    if pg is not None:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
