"""Standalone STFT roofline probe: >= 2048 signals (~1 GB traffic) per launch."""
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dl4ss_amd import ops  # noqa: E402


def run(n_sig, N, iters, complex_out):
    x = torch.randn(n_sig, N, device="cuda")
    T = ops.n_frames(N)
    Xc = torch.empty(n_sig, T, 129, 2, device="cuda") if complex_out else None
    mag = torch.empty(n_sig, T, 129, device="cuda")
    kw = dict(complex_out=complex_out, mag_out=True, out_c=Xc, out_mag=mag)
    for _ in range(5):
        ops.stft(x, **kw)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        ops.stft(x, **kw)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    per_sig = 4 * N + (12 if complex_out else 4) * T * 129
    gbs = n_sig * per_sig / (ms * 1e-3) / 1e9
    print(json.dumps({"kernel": "stft_fwd", "outputs": "complex+mag" if complex_out else "mag", "n_sig": n_sig,
                      "bytes_per_signal": per_sig, "ms": ms, "GB/s": gbs, "frac_8TBs": gbs / 8000}), flush=True)


def main(N=32000, iters=30):
    for n_sig in (2048, 4096):
        for c in (True, False):
            run(n_sig, N, iters, c)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "sweep":  # python tools/stft_bench.py sweep  (size sweep)
        for n in (512, 1024, 2048, 3072, 4096, 8192):
            run(n, 32000, 20, True)
    elif len(sys.argv) > 1:  # python tools/stft_bench.py N_SIG {mag|complex} ITERS  (profiling runs)
        run(int(sys.argv[1]), 32000, int(sys.argv[3]), sys.argv[2] == "complex")
    else:
        main()
