"""Time the step's GEMM shapes (B=32, T=251 BiLSTM-4L + Linear) through dl4ss_gemm.

  python tools/gemm_bench.py [bf16|fp32]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dl4ss_amd import ops  # noqa: E402

BT = 32 * 251
# (name, transA, transB, M, N, K, splitk, epilogue)
SHAPES = [
    ("fwd in-proj L0", False, True, BT, 2400, 129, 1, 0),
    ("fwd in-proj L1-3", False, True, BT, 2400, 600, 1, 0),
    ("fwd Linear+tanh", False, True, BT, 6450, 600, 1, 1),
    ("bwd dW_lin", True, False, 6450, 600, BT, 1, 0),
    ("bwd dH", False, False, BT, 600, 6450, 1, 0),
    ("bwd dW_ih L1-3", True, False, 2400, 600, BT, 4, 0),
    ("bwd dW_ih L0", True, False, 2400, 129, BT, 4, 0),
    ("bwd dW_hh (1 dir)", True, False, 1200, 300, BT, 4, 0),
    ("bwd dX", False, False, BT, 600, 2400, 1, 0),
]


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    dev = torch.device("cuda")
    total_ms = 0.0
    for name, ta, tb, M, N, K, sk, epi in SHAPES:
        A = torch.randn(*((K, M) if ta else (M, K)), device=dev)
        B = torch.randn(*((N, K) if tb else (K, N)), device=dev)
        C = torch.zeros(M, N, device=dev)
        bias = torch.randn(N, device=dev) if not ta else None
        sk = "auto" if epi == 0 else 1
        kw = dict(transA=ta, transB=tb, out=C, precision=prec, splitk=sk, bias=None, epilogue=epi, beta=0.0)
        for _ in range(3):
            ops.gemm(A, B, **kw)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        s.record()
        for _ in range(it):
            ops.gemm(A, B, **kw)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / it
        tf = 2.0 * M * N * K / (ms * 1e-3) / 1e12
        total_ms += ms
        print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "splitk": ops.auto_splitk(M, N, K) if sk == "auto" else 1,
                          "us": round(ms * 1e3, 1),
                          "TFLOP/s": round(tf, 1)}), flush=True)
    print(json.dumps({"precision": prec, "sum_us_one_each": round(total_ms * 1e3, 1)}))


if __name__ == "__main__":
    main()
