"""Time the step's GEMM shapes through dl4ss_gemm_bf16 (bf16 operands in HBM)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dl4ss_amd import ops  # noqa: E402
from gemm_bench import SHAPES  # noqa: E402


def main():
    if len(sys.argv) > 1:
        ops.GEMM_BF16_TARGET_WGS = int(sys.argv[1])
    tile = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    ops.gemm_bf16_set_tile(tile)
    dev = torch.device("cuda")
    total = 0.0
    for name, ta, tb, M, N, K, sk, epi in SHAPES:
        pad = lambda n: (n + 7) // 8 * 8  # producers write bf16 copies with 16-B aligned rows
        ra, ca = (K, M) if ta else (M, K)
        rb, cb = (N, K) if tb else (K, N)
        A = torch.randn(ra, pad(ca), device=dev).to(torch.bfloat16)[:, :ca]
        B = torch.randn(rb, pad(cb), device=dev).to(torch.bfloat16)[:, :cb]
        C = torch.zeros(M, N, device=dev)
        sk = "auto" if epi == 0 else 1
        kw = dict(transA=ta, transB=tb, out=C, splitk=sk, epilogue=epi, beta=0.0)
        for _ in range(3):
            ops.gemm_bf16(A, B, **kw)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        s.record()
        for _ in range(it):
            ops.gemm_bf16(A, B, **kw)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / it
        total += ms
        print(json.dumps({"gemm": name, "tile": tile, "wgs": ops.GEMM_BF16_TARGET_WGS, "M": M, "N": N, "K": K,
                          "us": round(ms * 1e3, 1),
                          "TFLOP/s": round(2.0 * M * N * K / (ms * 1e-3) / 1e12, 1)}), flush=True)
    print(json.dumps({"operands": "bf16", "sum_us_one_each": round(total * 1e3, 1)}))


if __name__ == "__main__":
    main()
