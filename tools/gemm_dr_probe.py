"""EXPERIMENT probe: the direct-to-register bf16 GEMM (tools/exp/gemm_dr.hip) against gemm_gl on the
step's GEMM shapes.  Build on the CPU first:  python tools/gemm_dr_probe.py build
On the GPU box:  python tools/gemm_dr_probe.py  -> one JSON line per (shape, kernel): us per launch and
max |err| / max |ref| against an fp32 matmul of the same bf16 operands."""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "exp", "gemm_dr.hip")
LIB = os.path.join(ROOT, "tools", "exp", "libgemm_dr.so")

# (name, M, N, K, the gemm_gl call's transB): C = A (M x K, k-contiguous) x Bt (N x K)^T
# (K padded to a multiple of 32 where the step's is not: the experiment kernel has no k tail)
SHAPES = [("dX", 8032, 600, 2400, False), ("inproj (K 608)", 8032, 2400, 608, True),
          ("linear (K 608)", 8032, 6450, 608, True), ("dH (K 6464)", 8032, 600, 6464, False)]
VARIANTS = {0: "4x4 tiles, 2 stages, 4 waves", 1: "4x4, 3 stages", 2: "4x4, 4 stages", 3: "2x4, 4 stages",
            4: "4x2, 4 stages", 5: "2x2, 6 stages", 6: "4x4, 3 stages, 1 wave per workgroup"}


def build():
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-shared", "-fPIC", SRC, "-o",
                    LIB], check=True)
    print(LIB)


def main():
    sys.path.insert(0, ROOT)
    import torch

    from dl4ss_amd import ops

    lib = ctypes.CDLL(LIB)
    lib.gemm_dr.argtypes = [ctypes.c_int] * 4 + [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                                                 ctypes.c_longlong, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p]
    g = torch.Generator(device="cuda").manual_seed(0)

    def timeit(fn, iters=30):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters * 1e3

    for name, M, N, K, tb in SHAPES:
        A = torch.randn(M, K, device="cuda", generator=g).bfloat16()
        Bt = torch.randn(N, K, device="cuda", generator=g).bfloat16()
        ref = A.float() @ Bt.float().T
        scale = ref.abs().max().item()
        C = torch.empty(M, N, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        flops = 2.0 * M * N * K
        B_gl = Bt if tb else Bt.T.contiguous()
        us = timeit(lambda: ops.gemm_bf16_gl(A, B_gl, transB=tb, out=C))
        err = (C - ref).abs().max().item() / scale
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "kernel": "gemm_gl", "us": us,
                          "tflops": flops / us / 1e6, "err": err}), flush=True)
        for v, desc in VARIANTS.items():
            def run():
                rc = lib.gemm_dr(v, M, N, K, A.data_ptr(), K, Bt.data_ptr(), K, C.data_ptr(), N, st)
                assert rc == 0, rc
            C.zero_()
            run()
            torch.cuda.synchronize()
            err = (C - ref).abs().max().item() / scale
            us = timeit(run)
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "kernel": f"dr{v}: {desc}", "us": us,
                              "tflops": flops / us / 1e6, "err": err}), flush=True)


if __name__ == "__main__":
    build() if len(sys.argv) > 1 and sys.argv[1] == "build" else main()
