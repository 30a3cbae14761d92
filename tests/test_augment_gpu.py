"""R1 augmentation on the GPU: ``dl4ss_mix_sources_rot`` (per-source rotation by the
AUGMENT_DATA shift after the normalisation, before the zero-padding) against the oracle's
fp32 restatement of the kernel arithmetic (``oracle.dsp.mix_sources_f32``) -- BIT-EXACT for the
rotated sources and the mixture, shifts 0, 1, len-1, len/2 and random, ragged lengths -- and
against the fp64 reference semantics (``dsp.normalise_source(..., shift)``, pinned to the
reference by tests/test_augment_cpu.py) within fp32 rounding."""
import numpy as np
import pytest
import torch

from dl4ss_amd import ops, synth
from oracle import dsp

pytestmark = pytest.mark.gpu


def _run(dev, raw, gains, lens, shifts):
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dt)).to(dev)
    s, m = ops.mix_sources(t(raw, np.float32), t(gains, np.float32), lengths=None if lens is None else t(lens, np.int32),
                           shifts=None if shifts is None else t(shifts, np.int32))
    torch.cuda.synchronize()
    return s.cpu().numpy(), m.cpu().numpy()


def test_rotation_bitwise_vs_oracle_ragged(dev):
    rng = np.random.default_rng(21)
    B, K, N = 4, 3, 4000
    raw = (rng.normal(0, 0.15, size=(B, K, N)) + 0.01).astype(np.float32)
    lens = np.array([[N, 2500, 1000], [N, N, N], [17, N - 1, 3999], [N, 1, 2]], np.int32)
    shifts = np.array([[0, 2499, 1], [N - 1, N // 2, 1], [16, 0, 1234], [int(rng.integers(0, N)), 0, 1]], np.int32)
    gains = rng.uniform(0.6, 1.8, size=(B, K)).astype(np.float32)
    s, m = _run(dev, raw, gains, lens, shifts)
    es, em = dsp.mix_sources_f32(raw, gains, lens, shifts)
    assert np.array_equal(s, es) and np.array_equal(m, em)
    # the same as the unrotated kernel output rolled within each source's length (index work exact)
    s0, _ = _run(dev, raw, gains, lens, None)
    for b in range(B):
        for k in range(K):
            ln, sh = int(lens[b, k]), int(shifts[b, k])
            assert np.array_equal(s[b, k, :ln], np.roll(s0[b, k, :ln], -sh)) and not s[b, k, ln:].any()
    # and the fp64 reference semantics (x -= mean; x /= max|x|; rotate; pad; gain; sum)
    for b in range(B):
        for k in range(K):
            ln = int(lens[b, k])
            if ln < 2:
                continue
            ref = dsp.normalise_source(raw[b, k, :ln], N, shift=int(shifts[b, k])) * float(gains[b, k])
            assert np.abs(s[b, k] - ref).max() < 2e-6


def test_rotation_full_size_bitwise(dev):
    """B = 32, K = 2, N = 32000 (the C2 shape) with random shifts, lengths = N."""
    gen = synth.SyntheticMixtures(n_samples=32000, k=2, seed=5)
    src, _, u = gen.batch(32)
    g = synth.gains_for(u, 2).astype(np.float32)
    rng = np.random.default_rng(5)
    shifts = rng.integers(0, 32000, size=(32, 2)).astype(np.int32)
    shifts[0] = (0, 31999)
    s, m = _run(dev, src.astype(np.float32), g, None, shifts)
    es, em = dsp.mix_sources_f32(src.astype(np.float32), g, None, shifts)
    assert np.array_equal(s, es) and np.array_equal(m, em)


def test_shift_zero_equals_unrotated_and_modulo(dev):
    rng = np.random.default_rng(2)
    raw = rng.normal(0, 0.2, size=(2, 2, 3000)).astype(np.float32)
    gains = np.ones((2, 2), np.float32)
    lens = np.array([[3000, 1500], [2999, 7]], np.int32)
    a = _run(dev, raw, gains, lens, np.zeros((2, 2), np.int32))
    b = _run(dev, raw, gains, lens, None)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    # a shift is taken modulo the source's own length (the reference draws s < len)
    c = _run(dev, raw, gains, lens, lens + np.array([[5, 3], [1, 2]], np.int32))
    d = _run(dev, raw, gains, lens, np.array([[5, 3], [1, 2]], np.int32))
    assert np.array_equal(c[0], d[0]) and np.array_equal(c[1], d[1])


def test_list_loader_train_split_rotates(dev, tmp_path):
    """wsj0list with augment=True: the batch carries one shift per source, drawn
    random.sample(range(len), 1)[0] in line order, and the features are the rotated mixture's."""
    import random

    from dl4ss_amd import wsj0list as wl
    from test_wsj0list_cpu import _dataset

    lst, data, _ = _dataset(tmp_path)
    N = 10000
    random.seed(3)
    (b,) = list(wl.ListBatches(lst, data, "train", batch=2, max_len=N, augment=True))
    random.seed(3)
    exp = [[random.sample(range(int(b["lengths"][r, k])), 1)[0] for k in range(2)] for r in range(2)]
    assert b["shifts"].tolist() == exp
    out = wl.features(b, dev)
    torch.cuda.synchronize()
    es, em = dsp.mix_sources_f32(b["raw"], b["gains"], b["lengths"], b["shifts"])
    assert np.array_equal(out["src"].cpu().numpy(), es) and np.array_equal(out["mix"].cpu().numpy(), em)
    ref = dsp.magnitude(em[0].astype(np.float64))
    assert np.abs(out["mix_mag"][0].cpu().numpy() - ref).max() < 1e-4 * ref.max()


def test_fromlist_loader_rotates_train_only(dev):
    """compat predata_fromList (C2 loader) under config_WSJ0_dB (AUGMENT_DATA = True,
    config_WSJ0_dB.py:112): train batches are drawn with shifts, valid batches are not."""
    import random

    from dl4ss_amd import compat
    from dl4ss_amd.compat import _data

    compat.install()
    import config_WSJ0_dB as c

    assert c.AUGMENT_DATA is True
    calls = []
    orig = _data.draw_shifts
    _data.draw_shifts = lambda L: (calls.append(np.asarray(L).shape), orig(L))[1]
    bs, ml = c.BATCH_SIZE, c.MAX_LEN
    c.BATCH_SIZE, c.MAX_LEN = 2, 4000
    try:
        import predata_fromList as pfl

        random.seed(1)
        d = next(pfl.prepare_data('once', 'train'))
        assert calls == [(2, 2)] and d["mix_wav"].shape == (2, 4000)
        next(pfl.prepare_data('once', 'valid'))
        assert calls == [(2, 2)]
    finally:
        _data.draw_shifts = orig
        c.BATCH_SIZE, c.MAX_LEN = bs, ml
