import json, sys, torch
sys.path.insert(0, '/root/repo') if False else None
sys.path.insert(0, __import__('os').environ.get('GRAFT_REPO_ROOT', '.'))
from dl4ss_amd import ops
dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(0)
dG = ops.to_bf16(torch.randn(8032, 2400, generator=g).to(dev))
W1 = ops.to_bf16(torch.randn(2400, 600, generator=g).to(dev))
dPre = ops.to_bf16(torch.randn(8032, 6456, generator=g).to(dev))
Wl = ops.to_bf16(torch.randn(6450, 600, generator=g).to(dev))
out = torch.empty(8032, 600, device=dev)
ws = torch.empty(200 << 20, device=dev, dtype=torch.uint8)
def t(fn):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20): fn()
    b.record(); torch.cuda.synchronize()
    return round(a.elapsed_time(b) * 50, 2)
res = {}
res["dX plain"] = t(lambda: ops.gemm_bf16_gl(dG, W1, out=out))
for gsz in (0, 480, 256, 384, 768, 1024):
    res[f"dX sk grid {gsz}"] = t(lambda: ops.gemm_bf16_gl_streamk(dG, W1, out, grid=gsz, ws=ws))
res["dH split3"] = t(lambda: ops.gemm_bf16_gl(dPre[:, :6450], Wl, out=out, splitk=3, ws=ws))
for gsz in (0, 256, 768):
    res[f"dH sk grid {gsz}"] = t(lambda: ops.gemm_bf16_gl_streamk(dPre[:, :6450], Wl, out, grid=gsz, ws=ws))
print(json.dumps(res))
