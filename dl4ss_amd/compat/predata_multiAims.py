"""Torch_multi/predata_multiAims.py restated on the GPU path -- the loader of the C1 driver
(``Torch_multi/main_run.py:11``: ``from predata_multiAims import prepare_data,
prepare_datasize, prepare_data_fake``).

Same generator contract as predata_multiAims_dB (:75-262: 'global' yields (sorted train
speakers, spk->idx, idx->spk, T, F, 32, n_spk), 'once' a batch dict forever) with the
plain mixing rule: every source mean-removed and peak-normalised, then summed at unit
gain (the dB branch at :177 is ``if 0 and ...``).  Imports ``config`` (Torch_multi/config.py).
"""
try:
    from . import predata_multiAims_dB as _dB
    from . import config
except ImportError:  # imported by its bare name (compat.install())
    import predata_multiAims_dB as _dB
    import config

channel_first = config.channel_first
prepare_datasize = _dB.prepare_datasize
prepare_data_fake = _dB.prepare_data_fake


def prepare_data(mode, train_or_test):
    return _dB.prepare_data(mode, train_or_test, gain_rule="none", cfg=config)
