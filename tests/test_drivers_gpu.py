"""The py3 driver mirrors (``dl4ss_amd/compat/drivers``) on the GPU: each driver's own
``train_step`` -- its module variants over ``myNet`` (HIP kernels), the reference's loop
lines, the HIP Adam of ``compat.optim`` -- run on the inputs and initial weights of the
reference-generated fixture of the same driver (``tests/golden/make_ref_fixtures.py``) and
compared with what the reference's own lines computed: loss, masks, masked predictions,
every gradient and the Adam-updated parameters (fp32 parity mode).  Plus short ``main()``
runs of the C2 loop (loader -> steps -> LR schedule) and the C5 recursive extraction."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import ref_recipe as rr  # noqa: E402

from dl4ss_amd import compat  # noqa: E402

pytestmark = pytest.mark.gpu

compat.install(drivers=True)

SPK = [f"spk{i:03d}" for i in range(101)]
D2I = {s: i for i, s in enumerate(SPK)}
I2D = {i: s for i, s in enumerate(SPK)}


def _train_data(fx):
    spk = fx["in/spk"]
    Y = fx["in/targets"]
    d = {"mix_feas": fx["in/mix_feas"],
         "multi_spk_fea_list": [{SPK[spk[b, k]]: Y[b, k] for k in range(spk.shape[1])} for b in range(spk.shape[0])]}
    if "in/mix_mag" in fx.files:
        d["mix_mag"] = fx["in/mix_mag"]
    return d


def _load(mods, fx):
    """mods: {prefix: module}; initial weights of the fixture's recipe."""
    specs = [(f"{p}.{n}", tuple(t.shape)) for p, m in mods.items() for n, t in m.state_dict().items()]
    w = rr.fixture_weights(fx, specs)
    for p, m in mods.items():
        m.load_state_dict({n: torch.from_numpy(w[f"{p}.{n}"]) for n in m.state_dict()})


def _grads_params(mods):
    g, p = {}, {}
    for pre, m in mods.items():
        for n, t in m.named_parameters():
            if t.grad is not None:
                g[f"{pre}.{n}"] = t.grad.detach().cpu().numpy()
            p[f"{pre}.{n}"] = t.detach().cpu().numpy()
    return g, p


def _check(fx, out, mods, tol_grad=2e-3, loss_key="loss"):
    lref = float(fx[f"out/{loss_key}"])
    assert abs(float(out["loss"]) - lref) <= 1e-4 * abs(lref), (float(out["loss"]), lref)
    mref = fx["out/mask"].astype(np.float64)
    mask = out["mask"].cpu().numpy().reshape(mref.shape)
    assert np.abs(mask - mref).max() <= 1e-4 * np.abs(mref).max()
    pref = fx["out/pred"].astype(np.float64)
    pred = out["pred"].cpu().numpy().reshape(pref.shape)
    assert np.linalg.norm(pred - pref) / np.linalg.norm(pref) < 1e-3
    g, p = _grads_params(mods)
    assert set(rr.unpack_names(fx, "grad")) <= set(g)
    bad = rr.check_params(fx, "grad", lambda n: g[n], tol_grad)
    assert not bad, bad
    bad = rr.check_adam(fx, lambda n: p[n])
    assert not bad, bad


def test_evalver_driver_step_matches_reference(dev):
    import main_run_sstune_EvalVer as drv

    fx = rr.load("ref_c2_evalver.npz")
    B, T, F = fx["in/mix_feas"].shape
    m, opt = drv.build(F, T, 101, 2)
    mods = {"mix": m["mix_hidden_layer_3d"], "emb": m["mix_speech_multiEmbedding"], "adj": m["adjust_layer"],
            "cls": m["mix_speech_classifier"]}
    _load(mods, fx)
    out = drv.train_step(m, opt, _train_data(fx), D2I, I2D, 101)
    assert [list(x) for x in out["top_k_mask_idx"]] == fx["out/top_k_idx"].tolist()
    _check(fx, out, {k: v for k, v in mods.items() if k != "cls"})
    assert all(t.grad is None for t in m["mix_speech_classifier"].parameters())  # discarded, no gradient


def test_crm_driver_step_matches_reference(dev):
    import main_run_sstune_cRM_EvalVer as drv

    fx = rr.load("ref_c3_crm.npz")
    B, T, F = fx["in/mix_feas"].shape
    m, opt = drv.build(F, T, 101, 2)
    mods = {"mix": m["mix_hidden_layer_3d"], "emb": m["mix_speech_multiEmbedding"], "adj": m["adjust_layer"]}
    _load(mods, fx)
    out = drv.train_step(m, opt, _train_data(fx), D2I, I2D, 101, run_classifier=False)
    _check(fx, out, mods, tol_grad=5e-3)


def test_main_run_driver_step_matches_reference(dev):
    import main_run as drv

    fx = rr.load("ref_c1_mainrun.npz")
    B, T, F = fx["in/mix_feas"].shape
    m, opt = drv.build(F, T, 101, 2, with_video=False)
    mods = {"mix": m["mix_hidden_layer_3d"], "emb": m["mix_speech_multiEmbedding"]}
    _load(mods, fx)
    out = drv.train_step(m, opt, _train_data(fx), D2I, 101, run_classifier=False)
    spk = fx["in/spk"]
    act = {"loss": out["loss"], "mask": torch.stack([out["mask"][b, spk[b]] for b in range(B)]),
           "pred": torch.stack([out["pred"][b, spk[b]] for b in range(B)])}
    inactive = np.ones(101, bool)
    inactive[spk.reshape(-1)] = False
    assert float(out["mask"][:, torch.from_numpy(inactive)].abs().max()) == 0.0
    _check(fx, act, mods)


def test_selfss_db_driver_step_matches_reference_3spk(dev):
    import main_run_multi_selfSS_dB as drv

    fx = rr.load("ref_c4_3spk.npz")
    B, T, F = fx["in/mix_feas"].shape
    m, opt = drv.build(F, T, 101, 3)
    mods = {"mix": m["mix_hidden_layer_3d"], "emb": m["mix_speech_multiEmbedding"]}
    _load(mods, fx)
    out = drv.train_step(m, opt, _train_data(fx), D2I, I2D, 101)
    _check(fx, out, mods)


def test_evalver_driver_main_loop(dev):
    """The C2 driver's main(): loader ('global' + 'once' batches of predata_fromList), steps,
    the 10-epoch LR halving on the HIP Adam's param_groups."""
    import config_WSJ0_dB as cfg
    import main_run_sstune_EvalVer as drv

    saved = (cfg.BATCH_SIZE, cfg.MAX_LEN, cfg.Load_param)
    cfg.BATCH_SIZE, cfg.MAX_LEN, cfg.Load_param = 2, 4000, False
    try:
        m, hist = drv.main(max_epoch=2, max_batches=2, log=lambda *a: None)
    finally:
        cfg.BATCH_SIZE, cfg.MAX_LEN, cfg.Load_param = saved
    assert len(hist) == 4 and all(np.isfinite(hist))


def test_grid_driver_recursive_extraction(dev):
    import config_WSJ0_dB as cfg
    import main_run_multi_selfSS_recuReal_GRID as drv

    # the Torch_multi loader this driver imports runs only with AUGMENT_DATA off
    # (predata_multiAims_dB.py:166, compat._data.torch_multi_augment)
    saved = (cfg.BATCH_SIZE, cfg.MAX_LEN, cfg.AUGMENT_DATA)
    cfg.BATCH_SIZE, cfg.MAX_LEN, cfg.AUGMENT_DATA = 1, 4000, False
    try:
        res = drv.main(max_batches=1, log=lambda *a: None)
    finally:
        cfg.BATCH_SIZE, cfg.MAX_LEN, cfg.AUGMENT_DATA = saved
    names = res[0][0]
    assert len(names) == 2 and names[0] is not None and names[0] != names[1]
