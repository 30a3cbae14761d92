"""Variant-library check: one eager + two graph training steps (default C2: B = 32, BiLSTM-4L, PIT, bf16) from a
fixed seed with the library named by DL4SS_LIB (default: the shipped one); writes SHA-256 digests of the
losses, the flat gradient and the updated parameters to argv[1] (JSON).  `--compare a b` reports whether two
such records are bitwise equal."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])


def run(out):
    from dl4ss_amd import engine, synth

    dev = torch.device("cuda")
    # LIB_BW_CFG="B,cell,L" (default the C2 step: 32,lstm,4)
    b_, cell, nl = os.environ.get("LIB_BW_CFG", "32,lstm,4").split(",")
    B, K, N = int(b_), 2, 32000
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=7)
    src, spk, u = gen.batch(B)
    batch = (torch.from_numpy(src.astype(np.float32)).to(dev),
             torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev),
             torch.from_numpy(spk.astype(np.int32)).to(dev))
    net = engine.SepNet(cell=cell, num_layers=int(nl), adjust=cell == "lstm", device=dev, seed=11)
    tr = engine.SepTrainer(net, B, K, N, mode="pit", precision="bf16")
    losses = [tr.step(*batch).clone()] + [tr.step_graph(*batch).clone() for _ in range(2)]
    tr.check()
    import hashlib
    import json
    rec = {k: hashlib.sha256(v.contiguous().view(torch.int32).cpu().numpy().tobytes()).hexdigest()
           for k, v in (("loss", torch.stack(losses)), ("grad", net.grad), ("flat", net.flat.detach()))}
    rec["loss_values"] = [float(x) for x in torch.stack(losses).flatten().cpu()]
    with open(out, "w") as f:
        json.dump(rec, f)


def compare(a, b):
    import json
    x, y = json.load(open(a)), json.load(open(b))
    ok = all(x[k] == y[k] for k in ("loss", "grad", "flat"))
    print("bitwise equal" if ok else "DIFFERENT", {k: x[k] == y[k] for k in ("loss", "grad", "flat")}, x["loss_values"])
    return ok


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    run(sys.argv[1])
