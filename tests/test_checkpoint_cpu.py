"""Reference checkpoint compatibility: the per-module params/param_* files of
EvalVer.py:677-690 (saved here in torch's legacy non-zip format, as torch-0.3 wrote them)
load into SepNet / ClassifierNet through the weights_only loader, and save back."""
import os

import numpy as np
import pytest
import torch

from dl4ss_amd import checkpoint, engine, infer
from oracle import model as om
from oracle import recursive as orc


def test_load_reference_module_files(tmp_path):
    torch.manual_seed(0)
    ref = om.SepModel(cell="lstm", num_layers=4)
    files = {}
    for kind, mod in (("hidden3d", ref.mix), ("emblayer", ref.emb), ("adjlayer", ref.adj)):
        p = str(tmp_path / f"param_mixdotadjust4lstmdot_WSJ0_{kind}_125")
        torch.save(mod.state_dict(), p, _use_new_zipfile_serialization=False)
        files[kind] = p
    net = engine.SepNet(cell="lstm", num_layers=4, device="cpu", seed=3)
    checkpoint.load_reference_params(net, **files)
    for name, t in ref.state_dict().items():
        assert torch.equal(net.view(name), t), name
    out = checkpoint.save_reference_params(net, str(tmp_path / "out"), "x", 5)
    net2 = engine.SepNet(cell="lstm", num_layers=4, device="cpu", seed=9)
    checkpoint.load_reference_params(net2, **out)
    assert torch.equal(net.flat, net2.flat)


def test_load_reference_classifier_drops_cnn_keys(tmp_path):
    torch.manual_seed(1)
    cls = orc.Classifier(129, 600, 3, 101)
    sd = dict(cls.state_dict())
    sd["cnn.weight"] = torch.zeros(3)  # EvalVer.py:547-549 pops keys containing 'cnn'
    p = str(tmp_path / "param_speech_2mix3lstm_best")
    torch.save(sd, p, _use_new_zipfile_serialization=False)
    cnet = infer.ClassifierNet(device="cpu")
    checkpoint.load_reference_classifier(cnet, p)
    for k, v in cls.state_dict().items():
        assert torch.equal(cnet.view(k), v), k


def test_strict_key_and_shape_errors(tmp_path):
    p = str(tmp_path / "bad")
    torch.save({"layer.weight_ih_l9": torch.zeros(2, 2)}, p)
    net = engine.SepNet(cell="gru", num_layers=2, device="cpu", adjust=False)
    try:
        checkpoint.load_reference_params(net, hidden3d=p)
        raise AssertionError("expected KeyError")
    except KeyError:
        pass
    torch.save({"layer.weight": torch.zeros(5, 5)}, p)
    try:
        checkpoint.load_reference_params(net, emblayer=p)
        raise AssertionError("expected ValueError")
    except ValueError:
        pass


LEGACY = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "legacy_py2_torch03")


def test_load_torch03_python2_legacy_files():
    """A torch-0.3 / Python-2 save (protocol-2 pickle, py2 str keys, LONG1 magic number,
    OrderedDict reduced from [key, value] pairs, 4-argument _rebuild_tensor over
    torch.cuda.FloatStorage on cuda:1; tests/golden/make_legacy_ckpt.py) loads through the
    weights_only path into a SepNet with the reference's key names (EvalVer.py:545-554)."""
    net = engine.SepNet(cell="gru", num_layers=2, hidden=8, emb=4, device="cpu", seed=1)
    files = {k: os.path.join(LEGACY, f"param_mix101_WSJ0_{k}_180") for k in ("hidden3d", "emblayer", "adjlayer")}
    checkpoint.load_reference_params(net, **files)
    exp = np.load(os.path.join(LEGACY, "expected.npz"))
    assert set(exp.files) == {n for n, _ in net.specs}
    for name in exp.files:
        assert torch.equal(net.view(name), torch.from_numpy(exp[name])), name
    # the raw file really is the legacy format: magic number pickle first, no zip header
    with open(files["hidden3d"], "rb") as f:
        head = f.read(4)
    assert head[:2] == b"\x80\x02" and head[2:3] == b"\x8a"


def test_strict_refuses_a_file_missing_net_parameters(tmp_path):
    """a 2-layer hidden3d file must not load into a 4-layer net under strict."""
    torch.manual_seed(0)
    small = om.SepModel(cell="lstm", num_layers=2)
    p = str(tmp_path / "param_x_hidden3d_1")
    torch.save(small.mix.state_dict(), p)
    net = engine.SepNet(cell="lstm", num_layers=4, device="cpu")
    with pytest.raises(KeyError, match="missing"):
        checkpoint.load_reference_params(net, hidden3d=p)
    checkpoint.load_reference_params(net, hidden3d=p, strict=False)  # explicit opt-out still works


def test_classifier_shape_mismatch_raises(tmp_path):
    cls = orc.Classifier(129, 300, 3, 101)  # H = 300 file into the H = 600 classifier
    p = str(tmp_path / "param_speech")
    torch.save(cls.state_dict(), p)
    with pytest.raises(ValueError, match="shape"):
        checkpoint.load_reference_classifier(infer.ClassifierNet(device="cpu"), p)
