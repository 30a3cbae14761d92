"""Reference-API mirror: py3 modules with the reference's import
names and call signatures, backed by the gfx950 kernels.

    from dl4ss_amd import compat
    compat.install()          # puts this directory first on sys.path
    import config, myNet, test_multi_labels_speech, bss_test
    from predata_multiAims_dB import prepare_data, prepare_datasize, prepare_data_fake
    from predata_fromList_cRM_123 import prepare_data as prepare_data_crm

A driver written against ``Torch_multi/main_run*.py`` / ``TDAA_beta/main_run_sstune_*``
swaps its in-file nn.Module definitions for ``from myNet import MIX_SPEECH, ...`` and
keeps its loop: feature extraction (mixing + STFT) and every module's forward and
backward run on the HIP path.  Data: there is no WSJ0 in this environment, so the
loaders draw seeded synthetic speech-shaped sources (``dl4ss_amd.synth``) for the
speakers of the reference's 101-speaker training split, with the reference's
mixing / gain rules and batch-dict contract.
"""
import os
import sys

PATH = os.path.dirname(os.path.abspath(__file__))


def install():
    """Make ``import config`` / ``import myNet`` / ... resolve to these modules."""
    if PATH not in sys.path:
        sys.path.insert(0, PATH)
    return PATH
