"""Diagnostic: the Linear + tanh -> bf16 V GEMM (8032 x 6450 x 600) with V's row pitch 6450 (the
step's contiguous (B, T*F, E) V) against pitches padded to 128-B multiples: is the epilogue paying
for partial cache-line writes?  HIP events around 20 launches; one JSON line per pitch."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from dl4ss_amd import ops  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(0)
X = ops.to_bf16(torch.randn(8032, 600, generator=g).to(dev))
Wl = ops.to_bf16(torch.randn(6450, 600, generator=g).to(dev))
bl = torch.randn(6450, device=dev)
for ld in (6450, 6456, 6464, 6528):
    Vb = torch.empty(8032, ld, device=dev, dtype=torch.bfloat16)
    out = Vb[:, :6450]

    def fn():
        ops.gemm_bf16_gl(X, Wl, transB=True, bias=bl, epilogue=ops.EPI_TANH_BF16, out=out)
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        fn()
    b.record()
    torch.cuda.synchronize()
    print(json.dumps({"ld": ld, "us": round(a.elapsed_time(b) * 50, 2)}), flush=True)
