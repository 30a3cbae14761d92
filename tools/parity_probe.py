"""Masked-magnitude (cRM: masked complex) rel-L2 of the HIP step against the CPU oracle at the
FULL sizes of the BASELINE configurations, per precision mode, and the C5 recursive extraction's
bf16 decision margins -- the measurements behind the per-config precision / parity table of
DESIGN.md section 6.  One JSON line per case.

  python tools/parity_probe.py [c1 c3 c4 c5 ...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dl4ss_amd import engine, synth  # noqa: E402
from oracle import model as om  # noqa: E402
from oracle import recursive as orc  # noqa: E402
from test_step_gpu import _oracle_features  # noqa: E402

MODES = [("bf16", "bf16"), ("bf16s", "bf16"), ("fp32", "bf16"), ("fp32", "fp32")]


def masked_rel(cell, L, B, K, N, mode, adjust, loss_channels=None, seed=3, modes=MODES):
    dev = torch.device("cuda", 0)
    torch.set_num_threads(16)
    net = engine.SepNet(cell=cell, num_layers=L, crm=mode == "crm", adjust=adjust, device=dev, seed=seed)
    ref = om.SepModel(cell=cell, num_layers=L, crm=mode == "crm", adjust=adjust)
    ref.load_state_dict({k: v.cpu() for k, v in net.state_dict().items()})
    src, spk, u = synth.SyntheticMixtures(n_samples=N, k=K, seed=seed).batch(B)
    gains = synth.gains_for(u, K)
    feats, X, Y = _oracle_features(src, gains, mode == "crm")
    with torch.no_grad():  # (C1's 101-channel loss changes the loss scale, not the K active masks)
        mask, *_ = ref(feats, torch.from_numpy(spk))
    if mode == "crm":
        pred_ref = om.loss_crm(mask, X, Y)[1]
    else:
        pred_ref = mask * X[:, None]
    for prec, rnn in modes:
        tr = engine.SepTrainer(net, B, K, N, mode=mode, precision=prec, rnn_precision=rnn, loss_channels=loss_channels)
        tr.spk.copy_(torch.from_numpy(spk.astype(np.int32)).to(dev))
        tr.features(torch.from_numpy(src.astype(np.float32)).to(dev), torch.from_numpy(gains.astype(np.float32)).to(dev))
        tr.forward()
        T, F = tr.T, tr.F
        pred = torch.empty((B, K, T * F, 2) if mode == "crm" else (B, K, T * F), device=dev)
        tr.attn(0, pred_out=pred)
        torch.cuda.synchronize()
        tr.check()
        p = pred.cpu().view(pred_ref.shape)
        rel = float((p - pred_ref).norm() / pred_ref.norm())
        print(json.dumps({"cell": cell, "L": L, "B": B, "K": K, "N": N, "mode": mode, "precision": prec,
                          "rnn_precision": rnn, "masked_rel_l2": rel, "finite": bool(torch.isfinite(p).all())}),
              flush=True)
        del tr
        torch.cuda.empty_cache()


def c5_margins(B, seed, thr=2e-2):
    from test_recursive_gpu import _feats, _models, _ours

    dev = torch.device("cuda", 0)
    torch.set_num_threads(16)
    mix, cls, emb = _models(seed)
    X = _feats(B, 32000, seed)
    T = X.shape[1]
    t0 = time.time()
    with torch.no_grad():
        ref = orc.recursive_extract(lambda x: mix(x), cls, emb.weight, X)
    t_ref = time.time() - t0
    for prec in (("bf16", "fp32") if B == 1 else ("bf16",)):  # (the fp32 classifier plan is B = 1 only)
        out = _ours(dev, mix, cls, emb, B, T, prec).run(X.to(dev))
        torch.cuda.synchronize()
        perr = [float((out["probs"][s].cpu() - ref["probs"][s]).abs().max()) for s in range(2)]
        agree = (out["spk"].cpu().long() == ref["spk"]).numpy()
        gaps = []
        for s in range(2):
            p = ref["probs"][s].sort(dim=1, descending=True).values
            gaps.append((p[:, 0] - p[:, 1]).numpy().tolist())
        merr = float((out["masks"].cpu() - ref["masks"]).abs().max())
        print(json.dumps({"config": "c5", "B": B, "seed": seed, "precision": prec, "prob_err_max": perr,
                          "ids_agree": agree.tolist(), "top12_gap": gaps, "mask_err_max": merr,
                          "t_oracle_s": t_ref}), flush=True)


def main():
    which = sys.argv[1:] or ["c4", "c3", "c1", "c5"]
    for w in which:
        if w == "c4":
            masked_rel("gru", 2, 32, 3, 32000, "label", adjust=False)
        elif w == "c3":
            masked_rel("gru", 2, 16, 2, 32000, "crm", adjust=True)
        elif w == "c1":
            masked_rel("gru", 2, 1, 2, 40000, "label", adjust=False, loss_channels=101)
        elif w == "c2":
            masked_rel("lstm", 4, 32, 2, 32000, "label", adjust=True)
        elif w == "c5":
            for B, seed in ((1, 11), (32, 7), (32, 3)):
                c5_margins(B, seed)


if __name__ == "__main__":
    main()
