"""dl4ss_amd: MI355X-native (gfx950 HIP) speech-separation training hot path.

STFT -> BiLSTM/BiGRU mask net -> label-ordered / PIT MSE -> cRM-apply + iSTFT,
re-designed for CDNA4 behind the reference's module/function API
(``config``, ``predata_*``, ``test_multi_labels_speech``, ``myNet``, ``bss_test``).
"""
__version__ = "0.1.0"
