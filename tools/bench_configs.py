"""Throughput of the other BASELINE.json configurations (bench.py measures C2, the headline).

  python tools/bench_configs.py [c1|c3|c4|c5 ...] [--steps K] [--warmup W] [--precision bf16|fp32]

  C1  Torch_multi/main_run.py: BiGRU-2L, B=1, 101-channel dense loss, no ADDJUST, N=40000 (5 s)
  C3  cRM path (main_run_sstune_cRM_EvalVer): BiGRU-2L, query width 2E, B=16, + the mask-apply
      iSTFT of the eval output (dl4ss_istft_apply) once per step
  C4  3-spk mixed SNR (predata_multiAims_3dB gains): BiGRU-2L, K=3, B=32
  C5  recursive extraction (GRID.py:383-475): classifier BiLSTM-3L H=600 + BiGRU-2L mask net,
      B=1 per replica, inference (2 extraction steps + final masks + iSTFT of both estimates);
      c5x32: 32 independent extractions batched per launch (rows never interact)

One JSON line per config: mixtures/s on one GPU (synthetic data, inputs resident in HBM).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dl4ss_amd import engine, infer, ops, synth  # noqa: E402


def _time(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps, out


def train_config(name, cell, L, B, K, N, mode, precision, steps, warmup, loss_channels=None, adjust=True,
                 eval_istft=False, emb_scale=1.0, rnn_precision=None):
    dev = torch.device("cuda")
    net = engine.SepNet(cell=cell, num_layers=L, crm=mode == "crm", adjust=adjust, device=dev, seed=1)
    if emb_scale != 1.0:  # the query embedding (N(0,1) rows at init) scaled: logits stay below saturation
        net.view("emb.layer.weight").mul_(emb_scale)
    tr = engine.SepTrainer(net, B, K, N, mode=mode, precision=precision, loss_channels=loss_channels,
                           rnn_precision=rnn_precision)
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=1)
    src, spk, u = gen.batch(B)
    raw = torch.from_numpy(src.astype(np.float32)).to(dev)
    gains = torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev)
    spk_d = torch.from_numpy(spk.astype(np.int32)).to(dev)
    T = tr.T
    y = torch.empty(B * K, 128 * (T - 1), device=dev) if eval_istft else None
    mask = torch.empty(B, K, T * tr.F, 2, device=dev) if eval_istft else None

    def step():
        loss = tr.step(raw, gains, spk_d)
        if eval_istft:  # cRM estimates -> waveforms (bss_eval_cRM, cRM_EvalVer.py:69-106)
            tr.attn(0, mask_out=mask)
            from dl4ss_amd import _lib
            _lib.call("dl4ss_istft_apply", _lib.ptr(tr.Xc_mix), _lib.ptr(mask), B * K, K, T, 1, 0, _lib.ptr(y),
                      _lib.stream_ptr())
        return loss

    losses = []

    def step_rec():
        loss = step()
        losses.append(loss[:1].clone())  # device copy: read after the timed window
        return loss

    dt, loss = _time(step_rec, steps, warmup)
    tr.check()
    timed = [float(x.item()) for x in losses[warmup:]]
    lv = timed[-1]
    r = {"config": name, "value": B / dt, "unit": "mixtures/s", "ms_per_step": dt * 1e3, "batch": B,
         "precision": precision, "rnn_precision": tr.rnn_precision, "loss": lv, "timed_losses": timed,
         "window_finite": bool(np.all(np.isfinite(timed))), "data": "synthetic", "n_gpus": 1}
    if emb_scale != 1.0:
        r["init"] = (f"query embedding scaled by {emb_scale} at init so every cRM logit stays below the 9.02 "
                     "saturation of the inverse compression in the timed window (the work per step does not "
                     "depend on the values)")
    if not np.isfinite(lv):  # reference-faithful: the cRM inverse compression is non-finite for logits >= 9.02
        r["note"] = "loss non-finite: cRM inverse compression saturates at |logit| >= 9.02 (SURVEY R11)"
    return r


def recursive_config(precision, steps, warmup, N=32000, B=1):
    dev = torch.device("cuda")
    net = engine.SepNet(cell="gru", num_layers=2, adjust=False, device=dev, seed=1)
    cnet = infer.ClassifierNet(129, 600, 3, 101, device=dev, seed=2)
    T = ops.n_frames(N)
    ex = infer.RecursiveExtractor(net, cnet, B, T, precision=precision)
    gen = synth.SyntheticMixtures(n_samples=N, k=2, seed=5)
    src, spk, u = gen.batch(B)
    raw = torch.from_numpy(src.astype(np.float32)).to(dev)
    gains = torch.from_numpy(synth.gains_for(u, 2).astype(np.float32)).to(dev)
    y = torch.empty(B * 2, 128 * (T - 1), device=dev)

    def extract():
        _, mix = ops.mix_sources(raw, gains)
        Xc, Xm = ops.stft(mix)
        out = ex.run(Xm)
        pred = out["masks"] * Xm[:, None]  # masked magnitudes of both estimates
        from dl4ss_amd import _lib
        _lib.call("dl4ss_istft_apply", _lib.ptr(Xc), _lib.ptr(pred.contiguous()), B * 2, 2, T, 0, 0, _lib.ptr(y),
                  _lib.stream_ptr())
        return out

    dt, out = _time(extract, steps, warmup)
    return {"config": f"C5: recursive extraction, classifier BiLSTM-3L H=600 + BiGRU-2L mask net, B={B} "
                      f"independent extractions per launch, N=32000",
            "value": B / dt, "unit": "mixtures/s", "ms_per_launch": dt * 1e3,
            "precision": precision, "speakers_row0": out["spk"][0].cpu().tolist(), "data": "synthetic", "n_gpus": 1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c1", "c3", "c4", "c5", "c5x32"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--precision", default="bf16", choices=["fp32", "bf16", "bf16s", "bf16s2", "mixed"],
                    help="c1/c3/c4: fp32, bf16, bf16s, bf16s2; c5: fp32, bf16, bf16s, mixed (infer.RecursiveExtractor)")
    ap.add_argument("--c5-precision", default=None, help="precision of the c5 configs (default: --precision)")
    ap.add_argument("--rnn-precision", default=None, choices=["fp32", "bf16"],
                    help="recurrent matvec precision (default: --precision)")
    a = ap.parse_args()
    rp = dict(rnn_precision=a.rnn_precision)
    for c in a.configs:
        if c == "c1":
            r = train_config("C1: BiGRU-2L, B=1, 101-channel loss, N=40000", "gru", 2, 1, 2, 40000, "label",
                             a.precision, a.steps, a.warmup, loss_channels=101, adjust=False, **rp)
        elif c == "c3":  # with the reference's N(0,1) query embedding the cRM logits saturate at init
            # (cRM_EvalVer.py:688: the loss is non-finite from the first steps, as in the reference);
            # the throughput is timed on a finite window (emb_scale) and reports every timed loss
            r = train_config("C3: cRM BiGRU-2L, B=16, N=32000, + mask-apply iSTFT", "gru", 2, 16, 2, 32000, "crm",
                             a.precision, a.steps, a.warmup, eval_istft=True, emb_scale=0.1, **rp)
        elif c == "c4":
            r = train_config("C4: 3-spk mixed SNR BiGRU-2L (no ADDJUST), B=32, N=32000", "gru", 2, 32, 3, 32000,
                             "label", a.precision, a.steps, a.warmup, adjust=False, **rp)
        elif c == "c5":  # the reference's replica: one mixture at a time
            r = recursive_config(a.c5_precision or a.precision, a.steps, a.warmup)
        elif c == "c5x32":  # 32 independent extractions (rows) per launch: the same latency-bound chain
            r = recursive_config(a.c5_precision or a.precision, a.steps, a.warmup, B=32)
        else:
            raise SystemExit(f"unknown config {c}")
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
