"""Where the bf16 step's masked-magnitude error comes from (CPU emulation, fp64 arithmetic with
bf16 rounding inserted at the points the HIP bf16 step rounds).  Points:

  feat   layer-0 features (dl4ss_f32_to_bf16)        wih    W_ih copies
  xin    inputs of layers >= 1 (bf16 layer outputs)  rec    recurrent matvec operands (W_hh, h_{t-1})
  lin    Linear operands (h_L, W_lin)                V      V = tanh(Linear) stored bf16
  linw / linh: only W_lin / only h_L of the Linear

usage: python tools/bf16_budget.py [C2|C4] [B]   -> one JSON line per rounding set
"""
import itertools
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from dl4ss_amd import engine, synth  # noqa: E402
from oracle import model as om  # noqa: E402
from test_step_gpu import _oracle_features  # noqa: E402


def bf(x, on):
    return x.to(torch.bfloat16).to(x.dtype) if on else x


def forward(sd, cell, L, feats, spk, adjust, R):
    x = bf(feats.double(), "feat" in R)
    B, T, _ = x.shape
    H = 300
    for l in range(L):
        outs = []
        for d, suf in enumerate(("", "_reverse")):
            Wih = bf(sd[f"mix.layer.weight_ih_l{l}{suf}"].double(), "wih" in R)
            Whh = bf(sd[f"mix.layer.weight_hh_l{l}{suf}"].double(), "rec" in R)
            bih = sd[f"mix.layer.bias_ih_l{l}{suf}"].double()
            bhh = sd[f"mix.layer.bias_hh_l{l}{suf}"].double()
            G = x @ Wih.t() + bih
            h = torch.zeros(B, H, dtype=torch.float64)
            c = torch.zeros(B, H, dtype=torch.float64)
            hs = [None] * T
            ts = range(T) if d == 0 else range(T - 1, -1, -1)
            for t in ts:
                gh = bf(h, "rec" in R) @ Whh.t() + bhh
                g = G[:, t]
                if cell == "lstm":
                    i, f, gg, o = g.add(gh).chunk(4, 1)
                    c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
                    h = torch.sigmoid(o) * torch.tanh(c)
                else:
                    ri, zi, ni = g.chunk(3, 1)
                    rh, zh, nh = gh.chunk(3, 1)
                    r = torch.sigmoid(ri + rh)
                    z = torch.sigmoid(zi + zh)
                    n = torch.tanh(ni + r * nh)
                    h = (1 - z) * n + z * h
                hs[t] = h
            outs.append(torch.stack(hs, 1))
        x = torch.cat(outs, 2)
        if l < L - 1:
            x = bf(x, "xin" in R)
    hL = x
    Wl = bf(sd["mix.Linear.weight"].double(), "lin" in R or "linw" in R)
    V = torch.tanh(bf(hL, "lin" in R or "linh" in R) @ Wl.t() + sd["mix.Linear.bias"].double())
    V = bf(V, "V" in R).view(B, T, 129, -1)
    q = sd["emb.layer.weight"].double()[torch.from_numpy(spk).long()]
    if adjust:
        m = hL.mean(1, keepdim=True).expand(B, q.shape[1], hL.shape[2])
        q = q + torch.cat([m, q], 2) @ sd["adj.layer.weight"].double().t()
    return torch.sigmoid(torch.einsum("btfe,bke->bktf", V, q))


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "C4"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    cfg = {"C2": ("lstm", 4, 2, True), "C4": ("gru", 2, 3, False)}[name]
    cell, L, K, adjust = cfg
    N = 32000
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    ref = om.SepModel(cell=cell, num_layers=L, adjust=adjust)
    torch.manual_seed(3)
    sd = {k: v.detach() for k, v in ref.state_dict().items()}
    src, spk, u = synth.SyntheticMixtures(n_samples=N, k=K, seed=3).batch(B)
    feats, X, Y = _oracle_features(src, synth.gains_for(u, K), False)
    truth = forward(sd, cell, L, feats, spk, adjust, set()) * X.double()[:, None]
    pts = ["feat", "wih", "xin", "rec", "lin", "V"]
    sets = [set()] + [{p} for p in pts] + [{"linw"}, {"linh"}, set(pts) - {"V"}, set(pts) - {"lin", "V"}, set(pts),
                                           {"xin", "rec", "linh"}, {"xin", "rec"}, {"xin", "rec", "linh", "feat"},
                                           {"xin", "rec", "linh", "V"}]
    if len(sys.argv) > 3:
        sets = [set(a.split(",")) for a in sys.argv[3:]]
    for R in sets:
        pred = forward(sd, cell, L, feats, spk, adjust, R) * X.double()[:, None]
        rel = float((pred - truth).norm() / truth.norm())
        print(json.dumps({"config": name, "B": B, "rounded": sorted(R), "masked_magnitude_rel_l2": rel}), flush=True)


if __name__ == "__main__":
    main()
