"""The reference import surface: every module name the five config
drivers import resolves after ``compat.install()``, and the py3 driver mirrors import and
expose the drivers' module variants.  Host-only (no kernel is called)."""
import importlib

import pytest

from dl4ss_amd import compat

# the non-stdlib, non-torch/numpy imports of each reference driver (file:line)
DRIVER_IMPORTS = {
    # Torch_multi/main_run.py:10-17
    "main_run": [("config", []), ("predata_multiAims", ["prepare_data", "prepare_datasize", "prepare_data_fake"]),
                 ("myNet", ["inception_v3"]), ("test_multi_labels_speech", ["multi_label_vector"]),
                 ("librosa", []), ("soundfile", [])],
    # TDAA_beta/main_run_sstune_EvalVer.py:10-22
    "main_run_sstune_EvalVer": [("config_WSJ0_dB", []), ("predata_fromList", ["prepare_data", "prepare_datasize"]),
                                ("test_multi_labels_speech", ["multi_label_vector"]), ("librosa", []),
                                ("soundfile", []), ("bss_test", ["cal"]), ("lrs", ["send"])],
    # TDAA_beta/main_run_sstune_cRM_EvalVer.py:10-17
    "main_run_sstune_cRM_EvalVer": [("config_WSJ0_dB", []),
                                    ("predata_fromList_cRM_123", ["prepare_data", "prepare_datasize"]),
                                    ("test_multi_labels_speech", ["multi_label_vector"]), ("librosa", []),
                                    ("soundfile", []), ("bss_test", ["cal"])],
    # Torch_multi/main_run_multi_selfSS_dB.py:10-21
    "main_run_multi_selfSS_dB": [("config_WSJ0_dB", []),
                                 ("predata_multiAims_dB", ["prepare_data", "prepare_datasize", "prepare_data_fake"]),
                                 ("myNet", []), ("test_multi_labels_speech", ["multi_label_vector"]),
                                 ("librosa", []), ("soundfile", []), ("bss_test", ["cal"])],
    # Torch_multi/main_run_multi_selfSS_recuReal_GRID.py:9-22
    "main_run_multi_selfSS_recuReal_GRID": [("config_WSJ0_dB", []), ("predata_multiAims_dB", ["prepare_data"]),
                                            ("myNet", []), ("test_multi_labels_speech", ["multi_label_vector"]),
                                            ("librosa", []), ("soundfile", []), ("bss_test", ["cal"])],
}


@pytest.mark.parametrize("driver", sorted(DRIVER_IMPORTS))
def test_every_driver_import_resolves(driver):
    compat.install()
    for mod, names in DRIVER_IMPORTS[driver]:
        m = importlib.import_module(mod)
        for n in names:
            assert hasattr(m, n), (driver, mod, n)


def test_librosa_and_soundfile_shims_only_when_absent():
    import sys

    compat.install()
    assert sys.path[-1] == compat.SHIMS  # appended last: an installed package would win
    import librosa
    import soundfile

    assert hasattr(librosa.core.spectrum, "stft") and hasattr(librosa.core.spectrum, "istft")
    assert hasattr(soundfile, "read") and hasattr(soundfile, "write")


DRIVER_MODULES = {
    "main_run": ["MIX_SPEECH", "MIX_SPEECH_classifier", "SPEECH_EMBEDDING", "ATTENTION", "VIDEO_QUERY", "top_k_mask",
                 "build", "train_step", "main"],
    "main_run_sstune_EvalVer": ["MIX_SPEECH", "MIX_SPEECH_classifier", "SPEECH_EMBEDDING", "ADDJUST", "ATTENTION",
                                "top_k_mask", "build", "load_params", "train_step", "main"],
    "main_run_sstune_cRM_EvalVer": ["MIX_SPEECH", "MIX_SPEECH_classifier", "SPEECH_EMBEDDING", "ADDJUST",
                                    "ATTENTION", "top_k_mask", "build", "train_step", "main", "cRM_k", "cRM_C"],
    "main_run_multi_selfSS_dB": ["MIX_SPEECH", "SPEECH_EMBEDDING", "ATTENTION", "top_k_mask", "build", "train_step",
                                 "main"],
    "main_run_multi_selfSS_recuReal_GRID": ["build", "load_params", "extract", "main"],
}


@pytest.mark.parametrize("driver", sorted(DRIVER_MODULES))
def test_driver_mirror_imports(driver):
    compat.install(drivers=True)
    m = importlib.import_module(driver)
    for n in DRIVER_MODULES[driver]:
        assert hasattr(m, n), (driver, n)


def test_evalver_module_variants_match_reference_shapes():
    """EvalVer.py:277-326: MIX_SPEECH is BiLSTM-4L returning (V, h); the classifier is
    BiLSTM-3L with hidden 2 HIDDEN_UNITS (state_dict shapes; constructed on the CPU)."""
    compat.install(drivers=True)
    import main_run_sstune_EvalVer as ev

    m = ev.MIX_SPEECH(129, 251)
    sd = m.state_dict()
    assert sd["layer.weight_ih_l0"].shape == (1200, 129) and "layer.weight_hh_l3_reverse" in sd
    assert m.return_hidden
    c = ev.MIX_SPEECH_classifier(129, 251, 101)
    sc = c.state_dict()
    assert sc["layer.weight_hh_l2"].shape == (2400, 600) and sc["Linear.weight"].shape == (101, 1200)


def test_inception_v3_constructs_with_reference_names():
    """myNet.inception_v3 / Inception3 construct (the reference's init raises, myNet.py:67) and
    carry exactly the reference Inception3's state_dict names and shapes
    (tests/golden/ref_inception_keys.npz, from Torch_multi/myNet.py itself)."""
    import os

    import numpy as np

    compat.install()
    import myNet

    net = myNet.inception_v3(pretrained=True)  # no local ImageNet file: random init
    sd = net.state_dict()
    fx = np.load(os.path.join(os.path.dirname(__file__), "golden", "ref_inception_keys.npz"))
    assert list(sd) == list(fx["names"])
    assert [",".join(map(str, v.shape)) for v in sd.values()] == list(fx["shapes"])
    assert net.transform_input


@pytest.mark.parametrize("driver", ["main_run_multi_selfSS_dB", "main_run_multi_selfSS_recuReal_GRID"])
def test_torch_multi_drivers_refuse_augment_at_start(driver):
    """config_WSJ0_dB.py:112 sets AUGMENT_DATA, which the Torch_multi loaders cannot run
    (predata_multiAims_dB.py:166 raises on the first source): the drivers on those loaders fail
    once, at start, with the fix in the message -- not inside their first batch."""
    compat.install(drivers=True)
    import config_WSJ0_dB as cfg

    m = importlib.import_module(driver)
    assert cfg.AUGMENT_DATA is True
    with pytest.raises(RuntimeError, match="AUGMENT_DATA = False"):
        m.main(log=lambda *a: None)
