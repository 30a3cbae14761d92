"""The deep-ring gemm_gl configurations (cfg 6: five 32-deep stages, cfg 7: four) against the shipped
128 x 128 double buffer (cfg 1) on the C2 step's GEMM shapes (B = 32: BT = 8032) and on the step's
grouped weight-gradient launch: us per launch (HIP events around 20 back-to-back launches, median of 5
such runs) and whether C is bitwise the cfg-1 result.  One JSON line per (shape, cfg, split)."""
import json
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from dl4ss_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda")
BT, H, F, E = 8032, 300, 129, 50
FE = F * E
g = torch.Generator(device="cpu").manual_seed(0)
CFGS = [int(c) for c in (sys.argv[1].split(",") if len(sys.argv) > 1 else "1,6,7".split(","))]
NOSIDE = "--no-side" in sys.argv


def rb(*shape):
    return ops.to_bf16(torch.randn(*shape, generator=g).to(dev))


def p8(n):
    return (n + 7) // 8 * 8


def timeit(fn, reps=20, runs=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(runs):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    return statistics.median(ts)


X0 = rb(BT, p8(F))
X0[:, F:] = 0
X1 = rb(BT, 2 * H)
W1 = rb(8 * H, 2 * H)
Wl = rb(FE, 2 * H)
dPre = rb(BT, p8(FE))
dPre[:, FE:] = 0
dG = [rb(BT, 8 * H) for _ in range(4)]
hp = [rb(BT, 2 * p8(H)) for _ in range(4)]
outs = [rb(BT, 2 * H) for _ in range(3)]
bias_in = torch.randn(8 * H, device=dev)
bias_l = torch.randn(FE, device=dev)
Vb = torch.empty(BT, FE, device=dev, dtype=torch.bfloat16)
G = torch.empty(BT, 8 * H, device=dev)
dH = torch.empty(BT, 2 * H, device=dev)
ws = torch.empty(64 << 20, device=dev, dtype=torch.uint8)

shapes = {
    "linear_tanh_bf16 8032x6450x600": (BT * FE * 600 * 2, dict(A=X1, B=Wl, transB=True, bias=bias_l,
                                                              epilogue=ops.EPI_TANH_BF16, out=Vb), (1,)),
    "inproj_l1 8032x2400x600": (BT * 2400 * 600 * 2, dict(A=X1, B=W1, transB=True, bias=bias_in, out=G), (1,)),
    "dX 8032x600x2400": (BT * 600 * 2400 * 2, dict(A=dG[0], B=W1, out=dH), (1, 2)),
    "dH 8032x600x6450": (BT * 600 * FE * 2, dict(A=dPre[:, :FE], B=Wl, out=dH), (1, 2, 3)),
}
for name, (flop, kw, splits) in shapes.items():
    kw = dict(kw)
    A, B, out = kw.pop("A"), kw.pop("B"), kw.pop("out")
    ref = None
    for split in splits:
        for cfg in CFGS:
            def f():
                ops.gemm_bf16_gl(A, B, out=out, splitk=split, ws=ws, **kw)
            _lib.call("dl4ss_gemm_gl_set_config", cfg)
            out.fill_(float("nan")) if out.dtype == torch.float32 else out.zero_()
            f()
            torch.cuda.synchronize()
            c = out.clone()
            if ref is None:
                ref = c
            same = bool(torch.equal(c.view(torch.int16) if c.dtype == torch.bfloat16 else c.view(torch.int32),
                                    ref.view(torch.int16) if ref.dtype == torch.bfloat16 else ref.view(torch.int32)))
            us = timeit(f)
            print(json.dumps({"shape": name, "cfg": cfg, "splitk": split, "us": round(us, 2),
                              "tflops": round(flop / us / 1e6, 1), "bitwise_equal_first": same}), flush=True)
_lib.call("dl4ss_gemm_gl_set_config", 0)

# the step's grouped weight-gradient launch (C2 with dW_lin on the side stream): dW_ih of the layers 3..0
# (unsplit), then both directions' dW_hh of every layer (split 4)
gW = [torch.zeros(8 * H, 2 * H if l else F, device=dev) for l in range(4)]
gH = [torch.zeros(8 * H, H, device=dev) for _ in range(4)]
probs = []
for l in (3, 2, 1, 0):
    xb = X0[:, :F] if l == 0 else outs[l - 1]
    probs.append(dict(A=dG[l], B=xb, out=gW[l], transA=True, transB=False, beta=0.0, splitk=1))
for l in (3, 2, 1, 0):
    for d in range(2):
        probs.append(dict(A=dG[l][:, d * 1200:(d + 1) * 1200], B=hp[l][:, d * p8(H):d * p8(H) + H],
                          out=gH[l][d * 1200:(d + 1) * 1200], transA=True, transB=False, beta=0.0, splitk=4))
flop = 2 * BT * (3 * 2400 * 600 + 2400 * F + 8 * 1200 * H)
ref = None
for cfg in [c for c in CFGS if c in (1, 2, 6, 7)]:
    grp = ops.GroupedGemm(probs, dev, cfg=cfg)
    for t in gW + gH:
        t.fill_(float("nan"))
    grp.run()
    torch.cuda.synchronize()
    c = torch.cat([t.flatten() for t in gW + gH])
    if ref is None:
        ref = c.clone()
    same = bool(torch.equal(c.view(torch.int32), ref.view(torch.int32)))
    us = timeit(grp.run)
    print(json.dumps({"shape": "grouped dW_ih x4 + dW_hh x8 (split 4)", "cfg": cfg, "us": round(us, 2),
                      "tflops": round(flop / us / 1e6, 1), "bitwise_equal_first": same}), flush=True)

# the side-stream dW_lin: persistent, 16 workgroups (cfg 2: 256 x 128 one per CU, the shipped form; the deep
# ring two per CU on 8 CUs' worth of slots x 2 = 16 / 32 workgroups)
dWl = torch.zeros(FE, 2 * H, device=dev)
rs = torch.zeros(FE, device=dev)
flop = 2 * BT * FE * 600
ref = None
for cfg, grid in ((2, 16), (6, 16), (6, 32), (7, 32)):
    if NOSIDE or (cfg not in CFGS and cfg != 2):
        continue
    grp = ops.GroupedGemm([dict(A=dPre[:, :FE], B=outs[2], out=dWl, transA=True, transB=False, beta=0.0, splitk=1,
                                rowsum=rs)], dev, grid=grid, cfg=cfg)
    dWl.fill_(float("nan"))
    grp.run()
    torch.cuda.synchronize()
    c = torch.cat([dWl.flatten(), rs])
    if ref is None:
        ref = c.clone()
    same = bool(torch.equal(c.view(torch.int32), ref.view(torch.int32)))
    us = timeit(grp.run, reps=3, runs=3)
    print(json.dumps({"shape": f"side dW_lin + rowsum grid {grid}", "cfg": cfg, "us": round(us, 2),
                      "tflops": round(flop / us / 1e6, 1), "bitwise_equal_first": same}), flush=True)
