"""Forward GEMM shapes of the step (input projection 8032x2400x600 + bias, Linear
8032x6450x600 + tanh): gemm_bb (the in-step kernel) vs hipBLASLt without the epilogue."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dl4ss_amd import ops  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    dev = torch.device("cuda")
    for name, M, N, K in (("in_proj", 8032, 2400, 600), ("linear", 8032, 6450, 600), ("in_proj_l0", 8032, 2400, 129)):
        pk = (K + 7) // 8 * 8
        A = torch.randn(M, pk, device=dev).to(torch.bfloat16)[:, :K]
        W = torch.randn(N, pk, device=dev).to(torch.bfloat16)[:, :K]
        bias = torch.randn(N, device=dev)
        C = torch.empty(M, N, device=dev)
        r = {"gemm": name, "M": M, "N": N, "K": K}
        r["gemm_bb_bias_us"] = timeit(lambda: ops.gemm_bf16(A, W, transB=True, bias=bias, out=C)) * 1e3
        r["lt_nobias_us"] = timeit(lambda: ops.gemm_bf16_lt(A, W, C, transB=True)) * 1e3
        Ab, Wb = A.contiguous(), W.contiguous()
        r["torch_bf16out_us"] = timeit(lambda: torch.matmul(Ab, Wb.t())) * 1e3
        for k in list(r):
            if k.endswith("_us"):
                r[k.replace("_us", "_TFs")] = round(2.0 * M * N * K / (r[k] * 1e-6) / 1e12, 1)
                r[k] = round(r[k], 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
