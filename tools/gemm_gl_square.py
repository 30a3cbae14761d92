"""Calibration of gemm_gl against the guide's reference structures: square bf16 GEMMs (4096^3,
8192 x 8192 x 4096) on every gemm_gl tile configuration and on hipBLASLt, uniform random
[-1, 1) operands (cdna_hip_programming.md §5.4 rule 25).  HIP events around 20 launches; one
JSON line per (shape, path)."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from dl4ss_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda")


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


cfgs = [int(c) for c in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 2, 3]
for M, N, K in ((4096, 4096, 4096), (8192, 8192, 4096)):
    A = ops.to_bf16(torch.rand(M, K, device=dev) * 2 - 1)
    B = ops.to_bf16(torch.rand(N, K, device=dev) * 2 - 1)
    C = torch.empty(M, N, device=dev)
    flop = 2.0 * M * N * K
    ref = None
    for cfg in cfgs:
        def f(cfg=cfg):
            _lib.call("dl4ss_gemm_gl_set_config", cfg)
            ops.gemm_bf16_gl(A, B, transB=True, out=C)
        us = timeit(f)
        if ref is None:
            ref = C.clone()
        err = float((C - ref).abs().max())
        print(json.dumps({"shape": f"{M}x{N}x{K}", "path": f"gemm_gl cfg {cfg}", "us": round(us, 2),
                          "tflops": round(flop / us / 1e6, 1), "max_abs_diff_vs_first": err}), flush=True)
    _lib.call("dl4ss_gemm_gl_set_config", 0)
    us = timeit(lambda: torch.matmul(A, B.t()))
    print(json.dumps({"shape": f"{M}x{N}x{K}", "path": "torch_bf16_matmul (vendor reference)", "us": round(us, 2),
                      "tflops": round(flop / us / 1e6, 1)}), flush=True)
