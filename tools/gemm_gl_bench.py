"""Time the C2 step's GEMM shapes (B = 32: BT = 8032) on gemm_gl (LDS-DMA, gemm_gl.hip) in each
tile configuration, beside torch's bf16 matmul (the vendor library: a timing reference only,
bf16 output, epilogue-free shapes).  HIP events around 20 back-to-back launches on random data;
prints one JSON line per shape and path (us per launch, TFLOP/s)."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from dl4ss_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda")
BT, H, F, E = 8032, 300, 129, 50
FE = F * E
g = torch.Generator(device="cpu").manual_seed(0)


def rb(*shape):
    return ops.to_bf16(torch.randn(*shape, generator=g).to(dev))


def p8(n):
    return (n + 7) // 8 * 8


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


X0 = rb(BT, p8(F))
X0[:, F:] = 0
W0 = rb(4 * H * 2, p8(F))
W0[:, F:] = 0
X1 = rb(BT, 2 * H)
W1 = rb(8 * H, 2 * H)
Wl = rb(FE, 2 * H)
dPre = rb(BT, p8(FE))
dPre[:, FE:] = 0
dG = rb(BT, 8 * H)
hp = rb(BT, 2 * p8(H))
bias_in = torch.randn(8 * H, device=dev)
bias_l = torch.randn(FE, device=dev)
Vb = torch.empty(BT, FE, device=dev, dtype=torch.bfloat16)
G = torch.empty(BT, 8 * H, device=dev)
dH = torch.empty(BT, 2 * H, device=dev)
dWl = torch.zeros(FE, 2 * H, device=dev)
dWih = torch.zeros(8 * H, 2 * H, device=dev)
dWih0 = torch.zeros(8 * H, F, device=dev)
dWhh = torch.zeros(8 * H, H, device=dev)

shapes = {
    "inproj_l0 8032x2400x129": (BT * 2400 * F * 2, dict(A=X0[:, :F], B=W0[:, :F], transB=True, bias=bias_in, out=G)),
    "inproj_l1 8032x2400x600": (BT * 2400 * 600 * 2, dict(A=X1, B=W1, transB=True, bias=bias_in, out=G)),
    "linear_tanh_bf16 8032x6450x600": (BT * FE * 600 * 2, dict(A=X1, B=Wl, transB=True, bias=bias_l,
                                                              epilogue=ops.EPI_TANH_BF16, out=Vb)),
    "dH 8032x600x6450": (BT * 600 * FE * 2, dict(A=dPre[:, :FE], B=Wl, out=dH)),
    "dW_lin 6450x600x8032": (BT * 600 * FE * 2, dict(A=dPre[:, :FE], B=X1, transA=True, out=dWl, beta=1.0)),
    "dX 8032x600x2400": (BT * 600 * 2400 * 2, dict(A=dG, B=W1, out=dH)),
    "dW_ih 2400x600x8032": (BT * 600 * 2400 * 2, dict(A=dG, B=X1, transA=True, out=dWih, beta=1.0)),
    "dW_ih0 2400x129x8032": (BT * 129 * 2400 * 2, dict(A=dG, B=X0[:, :F], transA=True, out=dWih0, beta=1.0)),
}
for name, (flop, kw) in shapes.items():
    A, B, out = kw.pop("A"), kw.pop("B"), kw.pop("out")
    ta, tb = kw.get("transA", False), kw.get("transB", False)
    epi = kw.get("epilogue", ops.EPI_NONE)
    beta = kw.get("beta", 0.0)
    SPLIT = {"dH": 3, "dW_lin": 2, "dX": 1, "dW_ih": 4, "dW_ih0": 4}.get(name.split()[0], 1)

    def gl(cfg, split=None):
        def f():
            _lib.call("dl4ss_gemm_gl_set_config", cfg)
            ops.gemm_bf16_gl(A, B, out=out, splitk=SPLIT if split is None else split, **kw)
        return f
    paths = {"gemm_gl": gl(1), "gemm_gl_256x128": gl(2), "gemm_gl_pp256": gl(4), "gemm_gl_pp256_10": gl(5)}
    if SPLIT > 1:
        paths["gemm_gl_256x128_halfsplit"] = gl(2, max(1, SPLIT // 2))
    for s in (2, 3, 4, 6, 8, 12):
        paths[f"gemm_gl_pp256 splitk={s}"] = gl(4, s)
        paths[f"gemm_gl_pp256_10 splitk={s}"] = gl(5, s)
    if epi == ops.EPI_NONE and kw.get("bias") is None:
        paths["torch_bf16_matmul"] = lambda: torch.matmul(A.t() if ta else A, B.t() if tb else B)
    for pname, fn in paths.items():
        try:
            us = timeit(fn)
            print(json.dumps({"shape": name, "path": pname, "us": round(us, 2), "tflops": round(flop / us / 1e6, 1)}),
                  flush=True)
        except RuntimeError as e:
            print(json.dumps({"shape": name, "path": pname, "error": str(e)[:200]}), flush=True)
# dW_hh: both directions batched
flop = 2 * BT * 1200 * H * 2
fns = {"gemm_gl": lambda: ops.gemm_bf16_gl(dG[:, :1200], hp[:, :H], transA=True, out=dWhh[:1200], beta=1.0,
                                           splitk=8, batch=2, strideA=1200, strideB=p8(H), strideC=1200 * H,
                                           M=1200, N=H, K=BT),
       "gemm_gl_pp256 splitk=8": lambda: (_lib.call("dl4ss_gemm_gl_set_config", 4), ops.gemm_bf16_gl(
           dG[:, :1200], hp[:, :H], transA=True, out=dWhh[:1200], beta=1.0, splitk=8, batch=2, strideA=1200,
           strideB=p8(H), strideC=1200 * H, M=1200, N=H, K=BT), _lib.call("dl4ss_gemm_gl_set_config", 0)),
       "gemm_gl_pp256 splitk=12": lambda: (_lib.call("dl4ss_gemm_gl_set_config", 4), ops.gemm_bf16_gl(
           dG[:, :1200], hp[:, :H], transA=True, out=dWhh[:1200], beta=1.0, splitk=12, batch=2, strideA=1200,
           strideB=p8(H), strideC=1200 * H, M=1200, N=H, K=BT), _lib.call("dl4ss_gemm_gl_set_config", 0))}
_lib.call("dl4ss_gemm_gl_set_config", 0)
for pname, fn in fns.items():
    us = timeit(fn)
    print(json.dumps({"shape": "dW_hh 2x1200x300x8032", "path": pname, "us": round(us, 2),
                      "tflops": round(flop / us / 1e6, 1)}), flush=True)

# split-K sweep of gemm_gl on the backward shapes (deterministic slabs + reduce)
if "--sweep" in sys.argv:
    sweep = {
        "dH 8032x600x6450": (BT * 600 * FE * 2, lambda s: ops.gemm_bf16_gl(dPre[:, :FE], Wl, out=dH, splitk=s)),
        "dW_lin 6450x600x8032": (BT * 600 * FE * 2, lambda s: ops.gemm_bf16_gl(dPre[:, :FE], X1, transA=True, out=dWl,
                                                                                beta=1.0, splitk=s)),
        "dX 8032x600x2400": (BT * 600 * 2400 * 2, lambda s: ops.gemm_bf16_gl(dG, W1, out=dH, splitk=s)),
        "dW_ih 2400x600x8032": (BT * 600 * 2400 * 2, lambda s: ops.gemm_bf16_gl(dG, X1, transA=True, out=dWih,
                                                                               beta=1.0, splitk=s)),
        "dW_hh 2x1200x300x8032": (2 * BT * 1200 * H * 2, lambda s: ops.gemm_bf16_gl(
            dG[:, :1200], hp[:, :H], transA=True, out=dWhh[:1200], beta=1.0, splitk=s, batch=2, strideA=1200,
            strideB=p8(H), strideC=1200 * H, M=1200, N=H, K=BT)),
    }
    for name, (flop, fn) in sweep.items():
        for s in (1, 2, 3, 4, 6, 8):
            us = timeit(lambda: fn(s))
            print(json.dumps({"shape": name, "path": f"gemm_gl splitk={s}", "us": round(us, 2),
                              "tflops": round(flop / us / 1e6, 1)}), flush=True)
