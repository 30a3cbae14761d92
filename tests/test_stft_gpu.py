"""GPU parity of the STFT / iSTFT / mixing kernels against the CPU oracle."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle import dsp
from dl4ss_amd import ops, synth

pytestmark = pytest.mark.gpu


def _sig(n_sig, N, seed):
    rng = np.random.default_rng(seed)
    return rng.standard_normal((n_sig, N)).astype(np.float32)


@pytest.mark.parametrize("N", [32000, 40000, 2000, 300, 1000 * 3 + 77])
def test_stft_matches_oracle(dev, N):
    x = _sig(3, N, N)
    X, mag = ops.stft(torch.from_numpy(x).to(dev))
    T = dsp.n_frames(N)
    assert X.shape == (3, T, 129, 2) and mag.shape == (3, T, 129)
    X, mag = X.cpu().numpy(), mag.cpu().numpy()
    for i in range(3):
        S = dsp.stft_tf(x[i].astype(np.float64))
        scale = np.abs(S).max()
        assert np.abs(X[i, ..., 0] - S.real).max() < 2e-6 * scale
        assert np.abs(X[i, ..., 1] - S.imag).max() < 2e-6 * scale
        assert np.abs(mag[i] - np.abs(S)).max() < 2e-6 * scale


def test_stft_golden_fixture(dev):
    g = np.load(os.path.join(ROOT, "tests", "golden", "stft_golden.npz"))
    X, _ = ops.stft(torch.from_numpy(g["x"]).to(dev), mag_out=False)
    X = X.cpu().numpy()
    scale = np.sqrt(g["re"] ** 2 + g["im"] ** 2).max()
    assert np.abs(X[..., 0] - g["re"]).max() < 2e-6 * scale
    assert np.abs(X[..., 1] - g["im"]).max() < 2e-6 * scale


def test_stft_logmag_and_conj(dev):
    x = _sig(2, 4000, 5)
    xt = torch.from_numpy(x).to(dev)
    _, lm = ops.stft(xt, complex_out=False, log=True)
    Xc, _ = ops.stft(xt, mag_out=False, conj=True)
    for i in range(2):
        np.testing.assert_allclose(lm[i].cpu().numpy(), dsp.log_magnitude(x[i]), atol=2e-4)
        S = dsp.stft_tf(x[i].astype(np.float64), conj=True)
        np.testing.assert_allclose(Xc[i, ..., 1].cpu().numpy(), S.imag, atol=2e-4)


@pytest.mark.parametrize("off_c,off_m", [(0, 0), (1, 1), (0, 2), (1, 3)])
@pytest.mark.parametrize("flags", ["both", "complex", "mag", "logmag"])
def test_stft_outputs_at_unaligned_offsets(dev, off_c, off_m, flags):
    """The forward emits 16-B granules of each tile's contiguous output range; outputs
    placed at 8-B / 4-B offsets inside larger buffers must be written bit-identically to
    freshly allocated ones, and nothing outside the output range may be touched."""
    x = torch.from_numpy(_sig(5, 5077, 11)).to(dev)  # T = 40: a full and a ragged tile per signal
    kw = dict(complex_out=flags in ("both", "complex"), mag_out=flags != "complex", log=flags == "logmag")
    Xr, mr = ops.stft(x, **kw)
    T = ops.n_frames(x.shape[-1])
    n_c, n_m = 5 * T * 129, 5 * T * 129
    bc = torch.full((2 * n_c + 2 * off_c + 8,), float("nan"), device=dev)
    bm = torch.full((n_m + off_m + 8,), float("nan"), device=dev)
    oc = bc[2 * off_c:2 * off_c + 2 * n_c].view(5, T, 129, 2)
    om_ = bm[off_m:off_m + n_m].view(5, T, 129)
    ops.stft(x, out_c=oc if kw["complex_out"] else None, out_mag=om_ if kw["mag_out"] else None, **kw)
    torch.cuda.synchronize()
    if kw["complex_out"]:
        assert torch.equal(oc, Xr)
        assert torch.isnan(bc[:2 * off_c]).all() and torch.isnan(bc[2 * off_c + 2 * n_c:]).all()
    if kw["mag_out"]:
        assert torch.equal(om_, mr)
        assert torch.isnan(bm[:off_m]).all() and torch.isnan(bm[off_m + n_m:]).all()


def test_stft_frame_indices_bit_exact(dev):
    """An impulse at sample n must land exactly in the frames covering n."""
    N = 4000
    for n in [0, 1, 127, 128, 129, 2047, 3999]:
        x = np.zeros((1, N), np.float32)
        x[0, n] = 1.0
        _, mag = ops.stft(torch.from_numpy(x).to(dev), complex_out=False)
        m = mag[0].cpu().numpy()
        ref = dsp.magnitude(x[0])
        nz = np.nonzero(ref.max(axis=1) > 1e-6)[0].tolist()
        got = np.nonzero(m.max(axis=1) > 1e-6)[0].tolist()
        assert got == nz, (n, got, nz)


@pytest.mark.parametrize("T", [251, 313, 17, 2])
def test_istft_matches_oracle(dev, T):
    rng = np.random.default_rng(T)
    S = (rng.standard_normal((2, T, 129)) + 1j * rng.standard_normal((2, T, 129))).astype(np.complex64)
    Sd = torch.from_numpy(np.stack([S.real, S.imag], -1).astype(np.float32)).to(dev)
    y = ops.istft(Sd).cpu().numpy()
    for i in range(2):
        ref = dsp.istft(S[i].T)
        assert y.shape[1] == ref.shape[0] == 128 * (T - 1)
        np.testing.assert_allclose(y[i], ref, atol=2e-5 * np.abs(ref).max())


def test_stft_istft_round_trip_full_size(dev):
    x = torch.from_numpy(_sig(64, 32000, 9)).to(dev)
    X, _ = ops.stft(x, mag_out=False)
    y = ops.istft(X)
    assert torch.allclose(y, x, atol=1e-4)


def test_mix_sources_matches_oracle(dev):
    gen = synth.SyntheticMixtures(n_samples=32000, k=2, seed=3)
    src, spk, u = gen.batch(4)
    g = synth.gains_for(u, 2)
    osrc, omix = ops.mix_sources(torch.from_numpy(src.astype(np.float32)).to(dev),
                                 torch.from_numpy(g.astype(np.float32)).to(dev))
    osrc, omix = osrc.cpu().numpy(), omix.cpu().numpy()
    for b in range(4):
        srcs = [dsp.normalise_source(src[b, k].astype(np.float32), 32000) for k in range(2)]
        s, m = dsp.mix_sources(srcs, g[b])
        np.testing.assert_allclose(osrc[b], s, atol=1e-5)
        np.testing.assert_allclose(omix[b], m, atol=2e-5)


def test_step_stft_one_launch_equals_two(dev):
    """The trainer's magnitude-mode features: mixtures and scaled sources share one signal buffer
    and ONE STFT launch covers both (SepTrainer._stfts); bitwise the two separate launches."""
    from dl4ss_amd import engine

    B, K, N = 4, 3, 8000
    net = engine.SepNet(cell="gru", num_layers=2, device=dev, seed=3)
    tr = engine.SepTrainer(net, B, K, N, mode="pit", precision="bf16")
    assert tr.mix.data_ptr() == tr._sig.data_ptr() and tr.src.data_ptr() == tr._sig[B:].data_ptr()
    src, _, u = synth.SyntheticMixtures(n_samples=N, k=K, seed=4).batch(B)
    raw = torch.from_numpy(src.astype(np.float32)).to(dev)
    gains = torch.from_numpy(synth.gains_for(u, K).astype(np.float32)).to(dev)
    tr.features(raw, gains)
    torch.cuda.synchronize()
    _, m_mix = ops.stft(tr.mix.clone(), complex_out=False, mag_out=True)
    _, m_src = ops.stft(tr.src.reshape(B * K, N).clone(), complex_out=False, mag_out=True)
    torch.cuda.synchronize()
    assert torch.equal(tr.mag_mix, m_mix)
    assert torch.equal(tr.mag_src.reshape(B * K, tr.T, tr.F), m_src)


@pytest.mark.parametrize("N,log", [(32000, False), (8000 + 77, False), (32000, True)])
def test_stft_bf16_magnitude_copy(dev, N, log):
    """dl4ss_stft_fwd_ex's bf16 copy of the first n_bf16 signals' (log) magnitudes: bitwise
    dl4ss_f32_to_bf16_2d of the fp32 output (full and partial frame tiles, the Nyquist bin), the
    fp32 output unchanged, row padding and the rows of later signals untouched."""
    from dl4ss_amd import _lib

    g = torch.Generator().manual_seed(3)
    n_sig, n_bf = 5, 3
    x = torch.randn(n_sig, N, generator=g).to(dev)
    T = ops.n_frames(N)
    _, ref = ops.stft(x, complex_out=False, log=log)
    mb = torch.full((n_sig * T, 136), 7.0, device=dev, dtype=torch.bfloat16)  # sentinel
    _, mag = ops.stft(x, complex_out=False, log=log, out_bf16=mb, n_bf16=n_bf)
    assert torch.equal(mag, ref)
    want = torch.empty(n_bf * T, 136, device=dev, dtype=torch.bfloat16)
    src = ref[:n_bf].reshape(n_bf * T, 129)
    _lib.call("dl4ss_f32_to_bf16_2d", _lib.ptr(src), 129, n_bf * T, 129, _lib.ptr(want), 136, _lib.stream_ptr())
    assert torch.equal(mb[:n_bf * T, :129], want[:, :129])
    assert (mb[:n_bf * T, 129:] == 7.0).all() and (mb[n_bf * T:] == 7.0).all()
