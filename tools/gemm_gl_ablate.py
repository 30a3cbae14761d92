"""Diagnostic: time gemm_gl on the input-projection and dW_ih shapes in the shipped library and
in ablation builds given by DL4SS_LIB (tools/variant_lib.py no_mfma -DGGL_NO_MFMA, no_dma
-DGGL_NO_DMA): which part of the k-loop bounds the kernel."""
import json
import os
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from dl4ss_amd import ops  # noqa: E402

dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(0)
X = ops.to_bf16(torch.randn(8032, 600, generator=g).to(dev))
W = ops.to_bf16(torch.randn(2400, 600, generator=g).to(dev))
dG = ops.to_bf16(torch.randn(8032, 2400, generator=g).to(dev))
G = torch.empty(8032, 2400, device=dev)
dW = torch.zeros(2400, 600, device=dev)
Wl = ops.to_bf16(torch.randn(6450, 600, generator=g).to(dev))
bl = torch.randn(6450, device=dev)
Vb = torch.empty(8032, 6450, device=dev, dtype=torch.bfloat16)
W1 = ops.to_bf16(torch.randn(2400, 600, generator=g).to(dev))
dH = torch.empty(8032, 600, device=dev)
for name, fn in (("inproj 8032x2400x600", lambda: ops.gemm_bf16_gl(X, W, transB=True, out=G)),
                 ("dW_ih 2400x600x8032 split4", lambda: ops.gemm_bf16_gl(dG, X, transA=True, out=dW, beta=1.0, splitk=4)),
                 ("linear_tanh_bf16 8032x6450x600", lambda: ops.gemm_bf16_gl(X, Wl, transB=True, bias=bl,
                                                                             epilogue=ops.EPI_TANH_BF16, out=Vb)),
                 ("dX 8032x600x2400", lambda: ops.gemm_bf16_gl(dG, W1, out=dH))):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        fn()
    b.record()
    torch.cuda.synchronize()
    print(json.dumps({"lib": os.environ.get("DL4SS_LIB", "shipped"), "shape": name, "us": a.elapsed_time(b) * 50}))
