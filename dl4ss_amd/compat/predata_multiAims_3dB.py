"""Torch_multi/predata_multiAims_3dB.py restated on the GPU path -- the 3-speaker mixed-SNR
loader of config C4 (imports ``config_WSJ0_dB``).

Generator contract of predata_multiAims_dB (:96-280); gains (:124-137, :192-217): a
2-speaker mixture gets 10^(dB/20 U) on one random channel, a 3-speaker one (MAX_MIX == 3)
the normal / large / small gains 10^(dB/20 0.5) (first speaker), 10^(dB/20 (0.5 + 0.5 U))
(second), 10^(dB/20 0.5 U) (third).  Set MIN_MIX = MAX_MIX = 3 in config_WSJ0_dB for C4.
"""
try:
    from . import predata_multiAims_dB as _dB
    from . import config_WSJ0_dB as config
except ImportError:  # imported by its bare name (compat.install())
    import predata_multiAims_dB as _dB
    import config_WSJ0_dB as config

channel_first = config.channel_first
prepare_datasize = _dB.prepare_datasize
prepare_data_fake = _dB.prepare_data_fake


def prepare_data(mode, train_or_test):
    return _dB.prepare_data(mode, train_or_test, gain_rule="db3", cfg=config)
