"""Diagnostic: how the persistent recurrence's workgroups were spread over the XCDs in a training step.

Each packed-kernel launch counts its workgroups per XCD in the group-formation counters at the end of
its hand-off workspace (birnn.hip group_pk: 8 per-XCD counters + the overflow count).  Runs a few graph
steps of the C2 workload and prints, for every (pass, layer) workspace of the last step, the per-XCD
counts and how many workgroups overflowed their XCD (their groups span XCDs: write-through hand-offs).

  python tools/placement_probe.py [steps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from dl4ss_amd import engine, ops, synth  # noqa: E402


def ctl_offset(B, H, plan):
    BC, NG, nchunk = plan["BC"], plan["NG"], plan["nchunk"]
    groups = 2 * nchunk
    HG = ((H + 1) // 2 + 1) & ~1
    fwd = max(groups * 2 * BC * H * 8, groups * 4 * BC * NG * 8 * 8)
    bwd = max(groups * 2 * NG * BC * H * 8, groups * 4 * NG * BC * HG * 8)
    n = max(fwd, bwd)
    return (n + 255) // 256 * 256


def main(steps=3):
    dev = torch.device("cuda")
    B, K, N = 32, 2, 32000
    net = engine.SepNet(cell="lstm", num_layers=4, device=dev, seed=1)
    tr = engine.SepTrainer(net, B, K, N, mode="pit", precision="bf16")
    src, spk, u = synth.SyntheticMixtures(n_samples=N, k=K, seed=1).batch(B)
    batch = (torch.from_numpy(src.astype(np.float32)).to(dev),
             torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev),
             torch.from_numpy(spk.astype(np.int32)).to(dev))
    tr.step(*batch)
    for _ in range(steps):
        tr.step_graph(*batch)
    torch.cuda.synchronize()
    plan = ops.birnn_plan("lstm", B, net.H)
    off = ctl_offset(B, net.H, plan) // 4
    print(f"side stream {tr.side}, plan {plan}")
    for pas in (0, 1):
        for l in range(net.L):
            ws = tr._ws_slot(l, bool(pas)).view(torch.int32)
            c = ws[off:off + 9].cpu().tolist()
            print(f"{'bwd' if pas else 'fwd'} layer {l}: per-XCD {c[:8]} (sum {sum(c[:8])}), overflow {c[8]}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
