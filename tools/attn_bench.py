"""Time the fused attention + loss passes of the C2 step in isolation (bf16 V, B = 32, T = 251,
F = 129, E = 50, K = 2, PIT): the COST pass, pit_select and the GRAD pass on the step's own
buffers after one real forward.  HIP events around `reps` launches of each; one JSON line.

  python tools/attn_bench.py [reps]        (run under rocprofv3 --pmc for the counter breakdown)
"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from dl4ss_amd import _lib, engine, synth  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda")
    B, K, N = 32, 2, 32000
    net = engine.SepNet(cell="lstm", num_layers=4, device=dev, seed=1)
    tr = engine.SepTrainer(net, B, K, N, mode="pit", precision="bf16")
    src, spk, u = synth.SyntheticMixtures(n_samples=N, k=K, seed=1).batch(B)
    tr.spk.copy_(torch.from_numpy(spk.astype(np.int32)).to(dev))
    tr.features(torch.from_numpy(src.astype(np.float32)).to(dev),
                torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev))
    tr.forward()
    st = _lib.stream_ptr()

    def cost():
        tr.attn(0)
        _lib.call("dl4ss_pit_select", _lib.ptr(tr.part_loss), B, K, tr.nblk, _lib.ptr(tr.perm), st)

    def grad():
        tr.attn(1, tr.perm)

    out = {}
    for name, fn in (("cost+pit_select", cost), ("grad", grad)):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name + "_us"] = e0.elapsed_time(e1) * 1e3 / reps
    rows = B * tr.T * tr.F
    grad_bytes = rows * (2 * 50 + 2 * 50 + 4 * (1 + K))  # V bf16 in, dPre bf16 out, |X| and K targets
    out["grad_bytes"] = grad_bytes
    out["grad_TB/s"] = grad_bytes / (out["grad_us"] * 1e-6) / 1e12
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
