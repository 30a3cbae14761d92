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
# the reference sets AUGMENT_DATA = True here, but its augmentation line is a numpy
# broadcast error (predata_multiAims_dB.py:166): disabled in this build
AUGMENT_DATA = False
