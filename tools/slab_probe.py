"""Top-layer BPTT launch alone (C2 shape: B = 32, T = 251, H = 300, BiLSTM, bf16 packed) reading dOut as S
split-K slabs, us per launch (HIP events, median of 5 x 5 launches), for S = 1..4 and slab strides padded by
PAD floats (a probe build with -DDL4SS_EXP_ZS_PAD reads DL4SS_EXP_ZS_PAD per process: run once per pad)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from dl4ss_amd import _lib  # noqa: E402

dev = torch.device("cuda")
B, T, H = 32, 251, 300
NGH = 4 * H
PAD = int(os.environ.get("DL4SS_EXP_ZS_PAD", "0"))
g = torch.Generator().manual_seed(0)
G = (torch.randn(B, T, 2, NGH, generator=g) * 0.5).to(dev)
whh = (torch.randn(2, NGH, H, generator=g) / H ** 0.5).to(dev)
bhh = (torch.randn(2, NGH, generator=g) * 0.1).to(dev)
o = torch.empty(B, T, 2 * H, device=dev)
hp = torch.empty_like(o)
act = torch.empty(B, T, 2, 4 * H, device=dev)
cs = torch.empty(B, T, 2, H, device=dev)
ws = _lib.query("dl4ss_birnn_workspace_bytes", 0, B, H)
wsb = torch.zeros((ws + 7) // 8, dtype=torch.int64, device=dev)
st = torch.zeros(1, dtype=torch.int32, device=dev)
_lib.call("dl4ss_birnn_fwd", 0, 1, B, T, H, _lib.ptr(G), _lib.ptr(whh), _lib.ptr(bhh), _lib.ptr(o), _lib.ptr(hp),
          _lib.ptr(act), _lib.ptr(cs), _lib.ptr(wsb), ws, _lib.ptr(st), _lib.stream_ptr())
torch.cuda.synchronize()
zs = B * T * 2 * H + PAD
sl = torch.randn(4 * zs, generator=g).to(dev)
dGb = torch.empty(B * T, 2 * NGH, device=dev, dtype=torch.bfloat16)
dbi = torch.zeros(2 * NGH, device=dev)
dbh = torch.zeros(2 * NGH, device=dev)


def run(S):
    flags = ((S - 1) & 3) << 12
    _lib.call("dl4ss_birnn_bwd_ex", 0, 1 | flags, B, T, H, _lib.ptr(sl), None, _lib.ptr(whh), _lib.ptr(act),
              _lib.ptr(cs), _lib.ptr(hp), None, None, _lib.ptr(dGb), None, _lib.ptr(dbi), _lib.ptr(dbh),
              _lib.ptr(wsb), ws, _lib.ptr(st), _lib.stream_ptr())


for S in (1, 2, 3, 4):
    run(S)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(5):
            run(S)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / 5)
    assert int(st.item()) == 0
    print(json.dumps({"S": S, "pad_floats": PAD, "us": round(statistics.median(ts), 1)}), flush=True)
