import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
import test_kernels_gpu as tk
from dl4ss_amd import _lib, ops

dev = torch.device("cuda")
cell, B, T, H = "lstm", 2, 9, 40
rnn, x = tk._birnn_ref(cell, B, T, 23, H, 7)
x.requires_grad_(True)
ref, _ = rnn(x)
gout = torch.randn_like(ref)
(ref * gout).sum().backward()
r = tk._run_birnn_fwd(dev, cell, rnn, x.detach(), H)
print("fwd err", (r["out"].cpu().double() - ref.detach()).abs().max().item())
# reference dG via manual recurrence on G
NGH = r["NGH"]
G = r["G"].cpu().double().view(B, T, 2, NGH).clone().requires_grad_(True)
whh = torch.stack([rnn.weight_hh_l0, rnn.weight_hh_l0_reverse]).detach()
bhh = torch.stack([rnn.bias_hh_l0, rnn.bias_hh_l0_reverse]).detach()
out2 = tk._manual_birnn(cell, G, whh, bhh, H)
print("manual vs torch", (out2 - ref).abs().max().item())
(out2 * gout).sum().backward()
gout_d = gout.float().to(dev)
dG = torch.zeros(B * T, 2 * NGH, device=dev)
_lib.call("dl4ss_birnn_bwd", 0, 0, B, T, H, _lib.ptr(gout_d), None, _lib.ptr(r["whh"]), _lib.ptr(r["act"]),
          _lib.ptr(r["cs"]), _lib.ptr(r["hprev"]), _lib.ptr(dG), None, _lib.ptr(r["ws"]), r["wsn"],
          _lib.ptr(r["status"]), _lib.stream_ptr())
torch.cuda.synchronize()
print("status", r["status"].item())
print("dG err", (dG.cpu().double().view(B, T, 2, NGH) - G.grad).abs().max().item(), G.grad.abs().max().item())
dwih = ops.gemm(dG, r["xd"], transA=True).cpu().double()
ref_dwih = torch.cat([rnn.weight_ih_l0.grad, rnn.weight_ih_l0_reverse.grad])
print("dwih err", (dwih - ref_dwih).abs().max().item(), ref_dwih.abs().max().item())
dwih2 = G.grad.view(B * T, 2 * NGH).T @ x.detach().view(B * T, -1)
print("dwih(ref dG) err", (dwih2 - ref_dwih).abs().max().item())
print("whh equal?", (r["whh"].cpu().double() - whh.view(2 * NGH, H)).abs().max().item())
ours = dG.cpu().double().view(B, T, 2, NGH)
err = (ours - G.grad).abs()
for d in range(2):
    print("dir", d, "per-t max err:", [round(err[:, t, d].max().item(), 4) for t in range(T)])
    print("   per-gate:", [round(err[:, :, d, q * H:(q + 1) * H].max().item(), 4) for q in range(4)])
print("per-b:", [round(err[b].max().item(), 4) for b in range(B)])
# same shapes, but with the per-step test's random weights
