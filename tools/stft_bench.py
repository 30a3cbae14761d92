"""Standalone STFT roofline probe: >= 2048 signals (~1 GB traffic) per launch."""
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dl4ss_amd import ops  # noqa: E402


def main(n_sig=2048, N=32000, iters=50):
    x = torch.randn(n_sig, N, device="cuda")
    T = ops.n_frames(N)
    Xc = torch.empty(n_sig, T, 129, 2, device="cuda")
    mag = torch.empty(n_sig, T, 129, device="cuda")
    for _ in range(5):
        ops.stft(x, out_c=Xc, out_mag=mag)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        ops.stft(x, out_c=Xc, out_mag=mag)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    per_sig = 4 * N + 12 * T * 129
    gbs = n_sig * per_sig / (ms * 1e-3) / 1e9
    print(json.dumps({"kernel": "stft_fwd", "n_sig": n_sig, "ms": ms, "GB/s": gbs, "frac_8TBs": gbs / 8000}))


if __name__ == "__main__":
    main()
