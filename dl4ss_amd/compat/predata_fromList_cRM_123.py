"""TDAA_beta/predata_fromList_cRM_123.py restated on the GPU path.

The reference reads WSJ0-mix list lines ``path dB path dB`` (regex at :158-163) and
yields False at the end of an epoch of ``batch_total`` batches.  With the list files
(``./create-speaker-mixtures/mix_{k}_spk_{tr,cv,tt}.txt``) and the wavs under
``config.aim_path/data`` present, the real mixtures are read (``dl4ss_amd.wsj0list``);
otherwise each line is a synthetic mixture with per-source dB drawn like the list files'
(uniform in [-2.5, 2.5] dB, the wsj0-2mix convention) and gains 10^(dB/20)
(:206-207,227-228).
'once' batches add the complex targets of the cRM path: mix_mag (B,T,F,2) =
convert2(STFT(mix)) (:255) and per-speaker (T,F,2) targets (:215-234).
"""
import random

import numpy as np

try:
    from . import config_WSJ0_dB as config
    from ._data import list_prepare_data
except ImportError:  # imported by its bare name (compat.install())
    import config_WSJ0_dB as config
    from dl4ss_amd.compat._data import list_prepare_data


def convert2(array):
    """(..., F) complex -> (..., F, 2) [re, im] float32 (predata_fromList_cRM_123.py:37-41)."""
    return np.stack([np.real(array), np.imag(array)], axis=-1).astype(np.float32)


def prepare_datasize(gen):
    data = next(gen)
    T, F = data["mix_feas"].shape[1:3]
    return T, F, 32, data["num_all_spk"], tuple(config.VideoSize)


def prepare_data(mode, train_or_test, min=None, max=None):
    """predata_fromList_cRM_123.py:90-293: list batches with complex targets, False at the
    end of the epoch (real WSJ0-mix lists when present, else synthetic lines)."""
    if min:
        config.MIN_MIX = min
    if max:
        config.MAX_MIX = max
    mix_k = random.sample(list(range(config.MIN_MIX, config.MAX_MIX + 1)), 1)[0]
    return list_prepare_data(config, mode, train_or_test, True, mix_k)
