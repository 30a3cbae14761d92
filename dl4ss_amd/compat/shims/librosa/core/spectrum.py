"""``librosa.core.spectrum.stft / istft`` on the HIP kernels (n_fft 256 / hop 128 only: the
reference's FRAME_LENGTH / FRAME_SHIFT, predata_*.py and EvalVer.py:64-65).  Orientation
is librosa's: stft returns (F, T) complex64, istft takes (F, T)."""
import numpy as np
import torch

from dl4ss_amd import ops


def stft(y, n_fft=256, hop_length=128, window="hann", center=True, **kwargs):
    if n_fft != 256 or hop_length != 128 or not center or (window not in ("hann", 256)):
        raise NotImplementedError("this build's STFT kernel is n_fft 256 / hop 128 / centred periodic Hann")
    x = torch.as_tensor(np.asarray(y, dtype=np.float32)).reshape(1, -1).cuda()
    Xc, _ = ops.stft(x, complex_out=True, mag_out=False)
    c = Xc[0].cpu().numpy()  # (T, F, 2)
    return np.ascontiguousarray((c[..., 0] + 1j * c[..., 1]).T.astype(np.complex64))


def istft(stft_matrix, hop_length=128, **kwargs):
    S = np.asarray(stft_matrix)
    if S.shape[0] != 129 or hop_length != 128:
        raise NotImplementedError("this build's iSTFT kernel is n_fft 256 / hop 128")
    St = np.ascontiguousarray(S.T)  # (T, F)
    c = torch.from_numpy(np.stack([St.real, St.imag], -1).astype(np.float32)).cuda()[None]
    return ops.istft(c)[0].cpu().numpy()
