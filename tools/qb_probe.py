"""Time dl4ss_query_bwd_ex by role (C2 shapes: B = 32, K = 2, D = 600, W = 50, 101 labels): each role alone
and all three (HIP events, 50 launches)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from dl4ss_amd import _lib  # noqa: E402

dev = torch.device("cuda")
B, K, D, W, T, NL = 32, 2, 600, 50, 251, 101
g = torch.Generator().manual_seed(0)
dq = torch.randn(B, K, W, generator=g).to(dev)
idx = torch.randint(0, NL, (B, K), generator=g, dtype=torch.int32).to(dev)
emb = torch.randn(NL, W, generator=g).to(dev)
wadj = torch.randn(W, D + W, generator=g).to(dev)
mean = torch.randn(B, D, generator=g).to(dev)
demb = torch.zeros(NL, W, device=dev)
dwadj = torch.zeros(W, D + W, device=dev)
dh = torch.zeros(B, D, device=dev)
P = _lib.ptr


def run(e, w, h):
    _lib.call("dl4ss_query_bwd_ex", P(dq), B, T, D, P(idx), P(emb), P(wadj), P(mean), K, W, P(demb) if e else None,
              P(dwadj) if w else None, P(dh) if h else None, NL, 0.0, _lib.stream_ptr())


for name, args in (("all", (1, 1, 1)), ("emb+zero", (1, 0, 0)), ("dW_adj", (0, 1, 0)), ("dh", (0, 0, 1))):
    run(*args)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(50):
        run(*args)
    b.record()
    torch.cuda.synchronize()
    print(name, round(a.elapsed_time(b) * 1e3 / 50, 2), "us")
