"""Reference-API mirror: py3 modules with the reference's import
names and call signatures, backed by the gfx950 kernels.

    from dl4ss_amd import compat
    compat.install()          # puts this directory first on sys.path
    import config, myNet, test_multi_labels_speech, bss_test
    from predata_multiAims_dB import prepare_data, prepare_datasize, prepare_data_fake
    from predata_fromList_cRM_123 import prepare_data as prepare_data_crm
    from predata_fromList import prepare_data        # C2 (EvalVer.py:11)
    from predata_multiAims import prepare_data       # C1 (main_run.py:11)
    from predata_multiAims_3dB import prepare_data   # C4 3-speaker gains
    import lrs, librosa, soundfile                   # lrs sink; librosa / soundfile shims if absent

Driver mirrors (``compat/drivers``, ``compat.install(drivers=True)``): py3 versions of the
reference's ``main_run.py`` (C1), ``main_run_sstune_EvalVer.py`` (C2),
``main_run_sstune_cRM_EvalVer.py`` (C3), ``main_run_multi_selfSS_dB.py`` (C4) and
``main_run_multi_selfSS_recuReal_GRID.py`` (C5), importing exactly the reference's module
names, with the driver's own module variants (e.g. EvalVer's BiLSTM-4L MIX_SPEECH returning
(V, h)) and the HIP Adam (``compat.optim``).

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


SHIMS = os.path.join(PATH, "shims")
DRIVERS = os.path.join(PATH, "drivers")


def install(shims=True, drivers=False):
    """Make ``import config`` / ``import myNet`` / ... resolve to these modules.

    ``shims``: also make ``import librosa`` / ``import soundfile`` work when those packages
    are absent (appended to the END of sys.path, so an installed package always wins): the
    reference drivers import both at the top (``main_run.py:16-17``).  ``drivers``: put the
    py3 driver mirrors (``compat/drivers``: ``main_run``, ``main_run_sstune_EvalVer``, ...)
    on the path too."""
    if PATH not in sys.path:
        sys.path.insert(0, PATH)
    if drivers and DRIVERS not in sys.path:
        sys.path.insert(1, DRIVERS)
    if shims and SHIMS not in sys.path:
        sys.path.append(SHIMS)
    return PATH
