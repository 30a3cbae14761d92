"""TDAA_beta/config_WSJ0_dB.py restated (constants; see config.py)."""
try:  # the reference module repeats config.py's constants
    from .config import *  # noqa: F401,F403
    from . import config as _base
except ImportError:  # imported by its bare name (compat.install())
    from config import *  # noqa: F401,F403
    import config as _base

is_ComlexMask = True
is_SelfTune = True
aim_path = '../Torch_multi/Dataset_Multi/' + str(_base.MODE) + '/' + _base.DATASET
MAX_EPOCH = 600
EPOCH_SIZE = 300
quchong_alpha = 1
dB = 5
# TDAA_beta/config_WSJ0_dB.py:111-112: set False, then True.  The list loaders
# (predata_fromList, predata_fromList_cRM_123) rotate every train source
# (dl4ss_mix_sources_rot); the Torch_multi loaders' form of the same line is a numpy
# broadcast error (predata_multiAims_dB.py:166) that this build raises as the reference
# does (compat._data.torch_multi_augment) -- run them with AUGMENT_DATA = False.
AUGMENT_DATA = True
