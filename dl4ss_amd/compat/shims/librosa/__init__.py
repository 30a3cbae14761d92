"""Minimal ``librosa`` for the driver mirrors when the real package is absent (it is, in
this image): ``librosa.core.spectrum.stft / istft`` with the conventions the reference
relies on (n_fft 256, hop 128, periodic Hann, centre + reflect padding, Σw² normalisation;
SURVEY section 8c), computed by the HIP kernels (dl4ss_stft_fwd / dl4ss_istft).  Only
installed by ``compat.install(shims=True)`` when ``import librosa`` would fail."""
from . import core  # noqa: F401
from .core.spectrum import istft, stft  # noqa: F401
