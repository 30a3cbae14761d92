"""Minimal ``soundfile`` for the driver mirrors when the real package is absent (it is, in
this image): ``read(path) -> (float64 samples, rate)`` and ``write(path, data, rate)``
over the RIFF/PCM reader-writer of ``dl4ss_amd.wsj0list`` -- the two calls the reference
makes (``predata_*.py`` reads, ``EvalVer.py:50,67-73`` writes).  Installed on sys.path only
by ``compat.install(shims=True)`` and only when ``import soundfile`` would fail."""
import numpy as np

from dl4ss_amd import wsj0list


def read(path, dtype="float64"):
    x, rate = wsj0list.read_wav(path)
    return np.asarray(x, dtype=dtype), rate


def write(path, data, samplerate, *args, **kwargs):
    wsj0list.write_wav(path, np.asarray(data, dtype=np.float64), samplerate)
