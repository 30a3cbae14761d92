"""Torch_multi/config.py restated (constants only; the reference's init_config() /
config.cfg machinery is never called by the Torch drivers)."""
import time

HAS_INIT_CONFIG = False
CONFIG_FILE = './config.cfg'
MODE = 1
DATASET = 'WSJ0'
aim_path = './Dataset_Multi/' + str(MODE) + '/' + DATASET
LOG_FILE_PRE = aim_path + '/dl4ss_output.' + time.strftime('%Y-%m-%d %H:%M:%S') + '.log'
TRAIN_LIST = aim_path + '/train_list'
VALID_LIST = aim_path + '/valid_list'
TEST_LIST = aim_path + '/test_list'
UNK_LIST = aim_path + '/unk_list'
Load_param = True
Save_param = True
Ground_truth = True
Comm_with_Memory = False
HIDDEN_UNITS = 300
NUM_LAYERS = 2
EMBEDDING_SIZE = 50
AUGMENT_DATA = False
MAX_EPOCH = 250
EPOCH_SIZE = 200
BATCH_SIZE = 16
BATCH_SIZE_EVAL = 10
FRAME_RATE = 8000
FRAME_LENGTH = int(0.032 * FRAME_RATE)  # 256
FRAME_SHIFT = int(0.016 * FRAME_RATE)   # 128
SHUFFLE_BATCH = True
MIN_MIX = 2
MAX_MIX = 2
ALPHA = 0.5
dB = 5
MAX_LEN = 5
MAX_LEN = FRAME_RATE * MAX_LEN
WINDOWS = FRAME_LENGTH
TMP_WEIGHT_FOLDER = aim_path + '/_tmp_weights'
UNK_SPK = False
UNK_SPK_SUPP = 3
START_EALY_STOP = 0
IS_LOG_SPECTRAL = False
ADD_BGD_NOISE = False
BGD_NOISE_WAV = None
BGD_NOISE_FILE = 'Dataset_Multi/BGD_150203_010_STR.CH1.wav'
Out_Sep_Result = True
VideoSize = (299, 299)
VIDEO_RATE = 10
channel_first = True

# ---- this build (not in the reference) ----
# mask net of MIX_SPEECH (main_run.py: BiGRU NUM_LAYERS; EvalVer: BiLSTM 4 layers)
MIX_CELL = 'gru'
# arithmetic of the HIP path: 'fp32' (parity) or 'bf16' (bf16 GEMM / recurrence operands)
PRECISION = 'fp32'
# synthetic speakers (no WSJ0 here): training split size = the reference's N_lab
NUM_SPEAKERS_TRAIN = 101
NUM_SPEAKERS_EVAL = 18
NUM_SPEAKERS_TEST = 18
DATA_SEED = 1
