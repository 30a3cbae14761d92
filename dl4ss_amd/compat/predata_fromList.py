"""TDAA_beta/predata_fromList.py restated on the GPU path -- the loader of the C2 driver
(``main_run_sstune_EvalVer.py:11``: ``from predata_fromList import prepare_data,
prepare_datasize``).

``prepare_data(mode, train_or_test)`` (:45-236): one WSJ0-mix list per split and mixture
size (``./create-speaker-mixtures/mix_{k}_spk_{tr,cv,tt}.txt``, :80-88); per line the
speakers, dB values and sample names come from the regexes at :113-115, every source is
cropped / mean-removed / peak-normalised / zero-padded and scaled by 10^(dB/20)
(:134-176), the mixture is their sum; 'global' yields (sorted train speakers, spk->idx,
idx->spk, T, F, 32, n_spk, batch_total) (:213-222), 'once' the batch dict with MAGNITUDE
targets (:223-234); after ``batch_total`` batches every ``next()`` yields ``False``
(:100-102).  Mixing and STFTs run on dl4ss_mix_sources(_ex) / dl4ss_stft_fwd; without the
list files and wavs (no WSJ0 here) the lines are synthetic (dB uniform in [-2.5, 2.5]).
"""
import random

try:
    from . import config_WSJ0_dB as config
    from ._data import list_prepare_data
except ImportError:  # imported by its bare name (compat.install())
    import config_WSJ0_dB as config
    from dl4ss_amd.compat._data import list_prepare_data

channel_first = config.channel_first


def prepare_datasize(gen):
    """predata_fromList.py:37-43 (the batch-dict form: (T, F, 32, n_spk, video size))."""
    data = next(gen)
    T, F = data["mix_feas"].shape[1:3]
    return T, F, 32, data["num_all_spk"], tuple(config.VideoSize)


def prepare_data(mode, train_or_test):
    mix_k = random.randint(config.MIN_MIX, config.MAX_MIX)  # :78
    return list_prepare_data(config, mode, train_or_test, False, mix_k)
