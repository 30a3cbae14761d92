"""Torch_multi/predata_multiAims_dB.py (and _3dB) restated on the GPU path.

``prepare_data(mode, train_or_test)`` is the reference's generator
(predata_multiAims_dB.py:75-262): 'global' yields (sorted train speakers,
spk->idx, idx->spk, T, F, 32, n_spk); 'once' yields a batch dict per
SURVEY Appendix A, forever.  Mixing: per-source mean removal + peak
normalisation, the 2-spk dB rule 10^(dB/20 U) on one random channel
(:124-130,177-190) or the 3-spk normal/large/small rule
(predata_multiAims_3dB.py:132-137,192-217), sum; features |STFT(mix)| (or
log|.| + eps with IS_LOG_SPECTRAL), complex mix_phase, clean magnitudes per
speaker -- all computed by dl4ss_mix_sources / dl4ss_stft_fwd.  Sources are the
synthetic speech-shaped stand-ins of dl4ss_amd.synth (no WSJ0 here).
"""
import random

import numpy as np

try:  # predata_multiAims_dB.py:7 imports config_WSJ0_dB as config
    from . import config_WSJ0_dB as config
    from ._data import BatchMaker, split_speakers, to_reference_dict
except ImportError:  # imported by its bare name (compat.install())
    import config_WSJ0_dB as config
    from dl4ss_amd.compat._data import BatchMaker, split_speakers, to_reference_dict

channel_first = True
GAIN_RULE = "db2"  # predata_multiAims_dB.py:124-130 (compat._data.gains_of)


def prepare_datasize(gen):
    """predata_multiAims_dB.py:55-61: (T, F, video frames, n_spk, video size) of one batch."""
    data = next(gen)
    if isinstance(data, dict):
        T, F = data["mix_feas"].shape[1:3]
        return T, F, 32, data["num_all_spk"], tuple(config.VideoSize)
    return data[1].shape[1], data[1].shape[2], data[4].shape[1], data[-1], (data[4].shape[2], data[4].shape[3])


def prepare_data_fake(train_or_test, num_labels):
    """predata_multiAims_dB.py:63-73: random arrays of the reference's fake shapes."""
    while True:
        out = []
        vid = (config.BATCH_SIZE, 32, 3, config.VideoSize[0], config.VideoSize[1]) if channel_first else \
            (config.BATCH_SIZE, 32, config.VideoSize[0], config.VideoSize[1], 3)
        for shp in [(config.BATCH_SIZE, 17040), (config.BATCH_SIZE, 134, 129), (config.BATCH_SIZE, 134, 129),
                    (config.BATCH_SIZE,), vid]:
            out.append(np.float32(np.random.random(shp)))
        out.append(num_labels)
        yield out


def prepare_data(mode, train_or_test, gain_rule=GAIN_RULE, cfg=None):
    """gain_rule / cfg: the variants predata_multiAims (unit gains, ``config``) and
    predata_multiAims_3dB (``config_WSJ0_dB``) share this generator."""
    cfg = cfg or config
    if cfg.MODE != 1 or cfg.DATASET != 'WSJ0':
        raise ValueError('No such dataset:{} for Speech.'.format(cfg.DATASET))
    all_spk_train = split_speakers(cfg, 'train')
    mix_k = random.randint(cfg.MIN_MIX, cfg.MAX_MIX)
    maker = BatchMaker(cfg, train_or_test, mix_k, seed_offset=random.randrange(1 << 20))
    while True:
        dev = maker.make(cfg.BATCH_SIZE, gain_rule=gain_rule, augment="torch_multi")
        if mode == 'global':
            spk = sorted(all_spk_train)
            d2i = {s: i for i, s in enumerate(spk)}
            i2d = {i: s for i, s in enumerate(spk)}
            T, F = dev["mix_mag"].shape[1:3]
            yield spk, d2i, i2d, T, F, 32, len(spk)
        elif mode == 'once':
            d = to_reference_dict(dev)
            d["num_all_spk"] = len(all_spk_train)
            yield d
