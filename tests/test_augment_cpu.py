"""R1 augmentation (config.AUGMENT_DATA) on CPU: the oracle pinned to the reference's own
statements (``tests/golden/ref_r1_augment.npz``, made by ``make_ref_fixtures.py r1`` from the
per-source blocks of TDAA_beta/predata_fromList.py:135-155, predata_fromList_cRM_123.py:183-203,
Torch_multi/predata_multiAims_dB.py:149-169 and predata_multiAims_3dB.py:164-184, executed with
the shift draw fixed), and the compat loaders' draw / error behaviour.  Bars: bit-exact (fp64
values, indices, error texts)."""
import random

import numpy as np
import pytest

from oracle import dsp
from dl4ss_amd.compat import _data

FX = None


def _fx():
    global FX
    if FX is None:
        import os

        FX = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_r1_augment.npz"))
    return FX


TAGS = ["fromlist", "fromlist_crm", "multiaims_db", "multiaims_3db"]


@pytest.mark.parametrize("tag", TAGS)
def test_oracle_preprocessing_matches_reference_bitwise(tag):
    fx = _fx()
    max_len = int(fx["r1/max_len"])
    guarded = bool(fx[f"r1/{tag}/guarded"])
    n_applied = n_err = 0
    for i in range(int(fx[f"r1/{tag}/count"])):
        key = f"r1/{tag}/{i}"
        x = fx[f"r1/sig/{int(fx[key + '/sig'])}"]
        aug, split, sh = bool(fx[key + "/aug"]), str(fx[key + "/split"]), int(fx[key + "/shift"])
        applied = aug and (split == "train" or not guarded)
        n = min(len(x), max_len)
        assert int(fx[key + "/drawn_from"]) == (n if applied else -1)  # random.sample(range(len(signal)), 1)
        err = str(fx[key + "/error"])
        try:
            got = dsp.normalise_source(x, max_len, shift=sh if applied else None, broadcast=not guarded)
        except ValueError as e:
            assert err and str(e) == err, (key, str(e), err)
            n_err += 1
            continue
        assert not err, (key, err)
        ref = fx[key + "/out"]
        assert got.dtype == ref.dtype and got.shape == ref.shape == (max_len,)
        assert np.array_equal(got, ref), key
        n_applied += applied
    assert n_applied >= 10
    # the Torch_multi broadcast form fails for every shift but 1, n-1 and n/2
    assert (n_err > 0) == (not guarded)


def test_list_rotation_is_a_rotation_of_the_unrotated_source():
    fx = _fx()
    max_len = int(fx["r1/max_len"])
    x = fx["r1/sig/1"]  # 625 samples: rotated over its own length, then zero-padded
    base = dsp.normalise_source(x, max_len)
    for s in (0, 1, 313, 624):
        r = dsp.normalise_source(x, max_len, shift=s)
        assert np.array_equal(r[:625], np.roll(base[:625], -s)) and not r[625:].any()


@pytest.mark.parametrize("tag", ["multiaims_db", "multiaims_3db"])
def test_torch_multi_loader_raises_like_reference(tag, monkeypatch):
    """compat._data.torch_multi_augment: the reference's ValueError text for the same draw."""
    fx = _fx()
    cfg = type("C", (), {"AUGMENT_DATA": True})
    seen = 0
    for i in range(int(fx[f"r1/{tag}/count"])):
        key = f"r1/{tag}/{i}"
        x = fx[f"r1/sig/{int(fx[key + '/sig'])}"]
        n = min(len(x), int(fx["r1/max_len"]))
        if not bool(fx[key + "/aug"]) or n != len(x):
            continue
        sh, err = int(fx[key + "/shift"]), str(fx[key + "/error"])
        monkeypatch.setattr(random, "sample", lambda pop, k, sh=sh: [sh])
        if err:
            with pytest.raises(ValueError) as e:
                _data.torch_multi_augment(cfg, n)
            assert str(e.value) == err
        else:  # the folded-sum cases: refused, not silently different data
            with pytest.raises(NotImplementedError):
                _data.torch_multi_augment(cfg, n)
        seen += 1
    assert seen >= 8
    cfg.AUGMENT_DATA = False
    assert _data.torch_multi_augment(cfg, 100) is None


def test_draw_shifts_follows_reference_draw_order():
    """One random.sample(range(len), 1)[0] per source, in line order (cRM_123.py:198-199)."""
    lens = np.array([[5, 7], [3, 11]])
    random.seed(7)
    got = _data.draw_shifts(lens)
    random.seed(7)
    exp = [[random.sample(range(5), 1)[0], random.sample(range(7), 1)[0]],
           [random.sample(range(3), 1)[0], random.sample(range(11), 1)[0]]]
    assert got.dtype == np.int32 and got.tolist() == exp


def test_mix_sources_f32_restatement_close_to_reference_semantics():
    """The kernel-precision restatement (fp32) against the fp64 reference semantics."""
    rng = np.random.default_rng(3)
    raw = rng.normal(0, 0.2, size=(2, 3, 900)).astype(np.float32)
    lens = np.array([[900, 600, 2], [900, 900, 450]])
    shifts = np.array([[0, 599, 1], [450, 1, 449]])
    gains = rng.uniform(0.5, 1.8, size=(2, 3)).astype(np.float32)
    src, mix = dsp.mix_sources_f32(raw, gains, lens, shifts)
    for b in range(2):
        ref = [dsp.normalise_source(raw[b, k, :lens[b, k]], 900, shift=int(shifts[b, k])) for k in range(3)]
        s, m = dsp.mix_sources(ref, gains[b])
        assert np.abs(src[b] - s).max() < 1e-6 and np.abs(mix[b] - m).max() < 2e-6
