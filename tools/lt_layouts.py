"""Diagnostic: hipBLASLt (dl4ss_gemm_bf16_lt, timed-candidate plans) on the step's
weight-gradient shapes in every operand layout: does a K-contiguous layout pay?

  python tools/lt_layouts.py      one JSON line per (shape, transA, transB)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from dl4ss_amd import ops  # noqa: E402

SHAPES = [("dW_ih L1-3", 2400, 600, 8032, 1), ("dW_ih L0", 2400, 136, 8032, 1), ("dW_hh", 1200, 300, 8032, 2),
          ("dW_lin", 6450, 600, 8032, 1)]


def main():
    dev = torch.device("cuda")
    for name, M, N, K, batch in SHAPES:
        for ta in (0, 1):
            for tb in (0, 1):
                A = torch.randn(batch, *((K, M) if ta else (M, K)), device=dev).to(torch.bfloat16)
                B = torch.randn(batch, *((N, K) if tb else (K, N)), device=dev).to(torch.bfloat16)
                C = torch.zeros(batch, M, N, device=dev)
                args = dict(transA=bool(ta), transB=bool(tb), beta=1.0, batch=batch, strideA=A[0].numel(),
                            strideB=B[0].numel(), strideC=C[0].numel())
                ops.gemm_bf16_lt(A[0], B[0], C[0], **args)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    ops.gemm_bf16_lt(A[0], B[0], C[0], **args)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / 20
                print(json.dumps({"gemm": name, "transA": ta, "transB": tb, "us": round(us, 1),
                                  "TFLOP/s": round(2 * M * N * K * batch / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
