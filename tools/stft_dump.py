"""Dump STFT outputs of the loaded library (DL4SS_LIB) for a bitwise comparison between builds:
python tools/stft_dump.py OUT.pt  (ragged lengths, offset views, the bf16 feature copy)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from dl4ss_amd import ops  # noqa: E402


def main(out):
    g = torch.Generator().manual_seed(7)
    res = {}
    for n_sig, N in ((3, 32000), (5, 4000), (2, 999), (7, 12345)):
        x = torch.randn(n_sig, N, generator=g).cuda()
        T = ops.n_frames(N)
        for off in (0, 1, 3):  # offset views: every alignment of the output rows
            Xc = torch.full((n_sig * T * 129 * 2 + 2 * off,), float("nan"), device="cuda")
            mg = torch.full((n_sig * T * 129 + off,), float("nan"), device="cuda")
            xc = Xc[2 * off:].view(n_sig, T, 129, 2)
            m = mg[off:].view(n_sig, T, 129)
            bf = torch.zeros(n_sig * T, 136, dtype=torch.bfloat16, device="cuda")
            ops.stft(x, complex_out=True, mag_out=True, out_c=xc, out_mag=m, out_bf16=bf, n_bf16=n_sig - 1)
            res[f"b{n_sig}_{N}_{off}"] = bf.view(torch.int16).cpu()
            res[f"c{n_sig}_{N}_{off}"] = Xc.cpu()
            res[f"m{n_sig}_{N}_{off}"] = mg.cpu()
        m2 = torch.empty(n_sig, T, 129, device="cuda")
        ops.stft(x, complex_out=False, mag_out=True, out_mag=m2, log=True)
        res[f"log{n_sig}_{N}"] = m2.cpu()
    torch.save(res, out)
    print("saved", len(res))


if __name__ == "__main__":
    main(sys.argv[1])
