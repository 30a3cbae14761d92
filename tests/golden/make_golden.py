"""Generates the committed golden fixtures from the CPU oracle (run from repo root:
``python tests/golden/make_golden.py``).  The reference itself is Python-2 code
that cannot run here, so these vectors are the oracle's own (parity pinned by
tests/test_oracle.py against numpy.fft / torch.nn / closed forms)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import dsp  # noqa: E402
from dl4ss_amd import synth  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    gen = synth.SyntheticMixtures(n_samples=2000, k=2, seed=7)
    src, spk, u = gen.batch(2)
    x = src.reshape(-1, 2000).astype(np.float32)
    re, im, yr = [], [], []
    for s in x:
        S = dsp.stft_tf(s.astype(np.float64))
        re.append(S.real)
        im.append(S.imag)
        yr.append(dsp.istft(S.T))
    np.savez_compressed(os.path.join(OUT, "stft_golden.npz"), x=x, re=np.array(re), im=np.array(im),
                        y_rec=np.array(yr))


if __name__ == "__main__":
    main()
