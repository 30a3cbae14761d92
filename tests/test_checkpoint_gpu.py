"""Reference checkpoints on the HIP path: the per-module
``params/param_*`` files of ``TDAA_beta/main_run_sstune_EvalVer.py:677-690`` (``_hidden3d_`` =
MIX_SPEECH, ``_emblayer_`` = SPEECH_EMBEDDING, ``_adjlayer_`` = ADDJUST) are loaded the way the
reference resumes from them (``EvalVer.py:545-554``: one ``load_state_dict(torch.load(path))``
per module) into BOTH the HIP ``SepNet`` on cuda (``checkpoint.load_reference_params``) and the
CPU oracle, one training step runs on each from the same synthetic batch, and loss, every
gradient and the Adam-updated parameters must agree at the fp32 parity bars of
``test_step_gpu._compare_step``.

Two sources of files:
* torch-0.3 / Python-2 files (protocol-2 pickle, ``torch.cuda.FloatStorage`` on ``cuda:1``)
  written by the same opcode-level writer that made the committed legacy fixture
  (``tests/golden/make_legacy_ckpt.py``; the committed fixture itself is H = 8, E = 4, checked on
  CPU by ``test_checkpoint_cpu.py``, while the fused attention kernel is built for the
  reference's E = 50), here at the reference's size: BiGRU-2L, H = 300, E = 50 with ADDJUST;
* C2-shaped files (BiLSTM-4L, H = 300, E = 50) written in torch's legacy non-zip format from
  a seeded oracle model -- the layout a reference training run leaves in ``params/``.
"""
import os

import numpy as np
import pytest
import torch

from dl4ss_amd import checkpoint, engine, synth
from oracle import model as om

from test_step_gpu import _oracle_features  # noqa: E402

pytestmark = pytest.mark.gpu

FILES = ("hidden3d", "emblayer", "adjlayer")


def _oracle_from_files(files, **kw):
    """EvalVer.py:545-554: each module's state_dict from its own file (weights_only here)."""
    ref = om.SepModel(**kw)
    ref.mix.load_state_dict(checkpoint.load_state(files["hidden3d"]))
    ref.emb.load_state_dict(checkpoint.load_state(files["emblayer"]))
    if ref.adj is not None:
        ref.adj.load_state_dict(checkpoint.load_state(files["adjlayer"]))
    return ref


def _step_from_files(dev, files, cell, L, H, E, B, K, N, mode):
    kw = dict(cell=cell, num_layers=L, hidden=H, emb=E)
    net = engine.SepNet(device=dev, seed=99, **kw)  # a different random init, overwritten by the files
    checkpoint.load_reference_params(net, **files)
    ref = _oracle_from_files(files, **kw)
    for name, p in ref.named_parameters():  # the load itself is exact
        assert torch.equal(net.view(name).cpu(), p.detach()), name
    tr = engine.SepTrainer(net, B, K, N, mode=mode, precision="fp32")
    src, spk, u = synth.SyntheticMixtures(n_samples=N, k=K, seed=17).batch(B)
    gains = synth.gains_for(u, K)
    feats, X, Y = _oracle_features(src, gains, False)
    opt = om.make_adam(ref)
    loss_ref, _, pred_ref = om.train_step(ref, opt, feats, X, Y, torch.from_numpy(spk), mode=mode)
    grads_ref = {n: p.grad.detach().clone() for n, p in ref.named_parameters()}
    tr.spk.copy_(torch.from_numpy(spk.astype(np.int32)).to(dev))
    tr.features(torch.from_numpy(src.astype(np.float32)).to(dev), torch.from_numpy(gains.astype(np.float32)).to(dev))
    tr.forward()
    pred = torch.empty(B, K, tr.T * tr.F, device=dev)
    tr.attn(0, pred_out=pred)
    loss = tr.loss_and_grad()
    tr.backward()
    tr.optimizer_step()
    tr.check()
    lv = float(loss[0].cpu())
    assert abs(lv - float(loss_ref)) <= 1e-4 * abs(float(loss_ref)), (lv, float(loss_ref))
    if mode == "label":
        rel = float((pred.cpu().view_as(pred_ref) - pred_ref).norm() / pred_ref.norm())
        assert rel < 1e-3, rel
    for name, gr in grads_ref.items():
        ours = net.view(name, net.grad).cpu()
        denom = float(gr.abs().max())
        err = float((ours - gr).abs().max()) / denom if denom > 0 else float(ours.abs().max())
        assert err < 2e-3, (name, err)
    for name, p in ref.named_parameters():  # Adam's first step: |update| <= ~lr everywhere
        assert float((net.view(name).cpu() - p.detach()).abs().max()) <= 2.1 * 2e-4, name
    return net


def test_legacy_torch03_files_drive_a_hip_step(dev, tmp_path):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_legacy_ckpt as mk

    mix, emb, adj = mk.module_dicts(H=300, E=50, layers=2, seed=4)
    for sd in (mix, adj):  # keep the gates off saturation at H = 300 (the writer's +-0.3 suits H = 8)
        for k in sd:
            sd[k] = sd[k] * 0.2
    files = {}
    for kind, sd in (("hidden3d", mix), ("emblayer", emb), ("adjlayer", adj)):
        files[kind] = str(tmp_path / f"param_mix101_WSJ0_{kind}_180")
        mk.write_state_dict(files[kind], sd)
        with open(files[kind], "rb") as f:  # the legacy format: protocol-2 pickle, LONG1 magic, no zip
            assert f.read(3) == b"\x80\x02\x8a"
    _step_from_files(dev, files, "gru", 2, 300, 50, 2, 2, 8000, "label")


@pytest.mark.parametrize("mode", ["label", "pit"])
def test_c2_reference_layout_files_drive_a_hip_step(dev, tmp_path, mode):
    torch.manual_seed(5)
    src = om.SepModel(cell="lstm", num_layers=4)
    files = {}
    for kind, mod in (("hidden3d", src.mix), ("emblayer", src.emb), ("adjlayer", src.adj)):
        p = str(tmp_path / f"param_mixdotadjust4lstmdot_WSJ0_{kind}_125")
        torch.save(mod.state_dict(), p, _use_new_zipfile_serialization=False)
        files[kind] = p
    net = _step_from_files(dev, files, "lstm", 4, 300, 50, 4, 2, 8000, mode)
    # and back out in the reference's layout: the updated weights round-trip exactly
    out = checkpoint.save_reference_params(net, str(tmp_path / "out"), "mix101", 126)
    again = engine.SepNet(cell="lstm", num_layers=4, device=dev, seed=3)
    checkpoint.load_reference_params(again, **out)
    assert torch.equal(again.flat, net.flat)
