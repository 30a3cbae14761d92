"""TDAA_beta/predata_fromList_cRM_123.py restated on the GPU path.

The reference reads WSJ0-mix list lines ``path dB path dB`` (regex at :158-163) and
yields False at the end of an epoch of ``batch_total`` batches; here each line is a
synthetic mixture with per-source dB drawn like the list files' (uniform in
[-2.5, 2.5] dB, the wsj0-2mix convention) and gains 10^(dB/20) (:206-207,227-228).
'once' batches add the complex targets of the cRM path: mix_mag (B,T,F,2) =
convert2(STFT(mix)) (:255) and per-speaker (T,F,2) targets (:215-234).
"""
import random

import numpy as np

try:
    from . import config_WSJ0_dB as config
    from ._data import BatchMaker, split_speakers, to_reference_dict
except ImportError:  # imported by its bare name (compat.install())
    import config_WSJ0_dB as config
    from dl4ss_amd.compat._data import BatchMaker, split_speakers, to_reference_dict

LINES_PER_EPOCH = {'train': 20000, 'valid': 5000, 'test': 3000}


def convert2(array):
    """(..., F) complex -> (..., F, 2) [re, im] float32 (predata_fromList_cRM_123.py:37-41)."""
    return np.stack([np.real(array), np.imag(array)], axis=-1).astype(np.float32)


def prepare_datasize(gen):
    data = next(gen)
    T, F = data["mix_feas"].shape[1:3]
    return T, F, 32, data["num_all_spk"], tuple(config.VideoSize)


def prepare_data(mode, train_or_test, min=None, max=None):
    if min:
        config.MIN_MIX = min
    if max:
        config.MAX_MIX = max
    all_spk_train = split_speakers(config, 'train')
    batch_total = LINES_PER_EPOCH.get(train_or_test, 3000) // config.BATCH_SIZE
    mix_number_list = list(range(config.MIN_MIX, config.MAX_MIX + 1))
    rng = np.random.default_rng(getattr(config, "DATA_SEED", 1))
    mix_k = random.sample(mix_number_list, 1)[0]
    makers = {}
    for _ in range(batch_total):
        maker = makers.setdefault(mix_k, BatchMaker(config, train_or_test, mix_k))
        db = rng.uniform(-2.5, 2.5, size=(config.BATCH_SIZE, mix_k))
        dev = maker.make(config.BATCH_SIZE, complex_targets=True, db_list=db)
        if mode == 'global':
            spk = sorted(all_spk_train)
            T, F = dev["mix_mag"].shape[1:3]
            yield spk, {s: i for i, s in enumerate(spk)}, {i: s for i, s in enumerate(spk)}, T, F, 32, len(spk), \
                batch_total
        elif mode == 'once':
            d = to_reference_dict(dev, complex_targets=True)
            d["num_all_spk"] = len(all_spk_train)
            d["batch_total"] = batch_total
            yield d
        mix_k = random.sample(mix_number_list, 1)[0]
    yield False
