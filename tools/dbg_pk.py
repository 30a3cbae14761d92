"""Debug: packed bf16 forward vs fp32 forward vs an fp64 recurrence (tests/_manual_birnn)."""
import sys, torch
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from dl4ss_amd import _lib
from test_kernels_gpu import _manual_birnn
dev = torch.device('cuda')
for B, T in [(3, 8), (32, 12)]:
    H = 300; NGH = 1200
    g = torch.Generator().manual_seed(B * 31 + T)
    G = torch.randn(B, T, 2, NGH, generator=g, dtype=torch.float64) * 0.5
    whh = torch.randn(2, NGH, H, generator=g, dtype=torch.float64) / H ** 0.5
    bhh = torch.randn(2, NGH, generator=g, dtype=torch.float64) * 0.1
    ref = _manual_birnn("lstm", G, whh, bhh, H, bf16=True)
    res = {}
    for prec in (0, 1):
        Gd, whd, bhd = G.float().to(dev).contiguous(), whh.float().to(dev).contiguous(), bhh.float().to(dev).contiguous()
        o = torch.zeros(B, T, 2 * H, device=dev); hp = torch.zeros_like(o)
        act = torch.zeros(B, T, 2, 4 * H, device=dev); cs = torch.zeros(B, T, 2, H, device=dev)
        ws = _lib.query("dl4ss_birnn_workspace_bytes", 0, B, H)
        wsb = torch.empty((ws + 7) // 8, dtype=torch.int64, device=dev)
        st = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.call("dl4ss_birnn_fwd", 0, prec, B, T, H, _lib.ptr(Gd), _lib.ptr(whd), _lib.ptr(bhd), _lib.ptr(o),
                  _lib.ptr(hp), _lib.ptr(act), _lib.ptr(cs), _lib.ptr(wsb), ws, _lib.ptr(st), _lib.stream_ptr())
        torch.cuda.synchronize()
        res[prec] = dict(o=o.cpu().double(), hp=hp.cpu(), act=act.cpu(), cs=cs.cpu(), st=int(st.item()))
        print(B, T, 'prec', prec, 'status', res[prec]['st'], 'o vs fp64 ref', float((res[prec]['o'] - ref).abs().max()))
    for k in ('o', 'hp', 'act', 'cs'):
        d = (res[0][k].float() - res[1][k].float()).abs()
        print(B, T, k, 'fp32 vs bf16 maxdiff', float(d.max()), 'at', [int(i) for i in torch.nonzero(d == d.max())[0]])
