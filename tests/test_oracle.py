"""Pins the CPU oracle against in-container independent references (the
reference ships no golden vectors for this path)."""
import numpy as np
import pytest
import torch

from oracle import dsp, model
from dl4ss_amd import synth


def test_frame_count_matches_reference_lengths():
    # EvalVer.py:49 hard-codes 39936 = 128 * (313 - 1) for MAX_LEN = 5 s
    assert dsp.n_frames(40000) == 313 and dsp.n_frames(32000) == 251
    S = dsp.stft(np.random.default_rng(0).standard_normal(40000))
    assert S.shape == (129, 313) and S.dtype == np.complex64
    assert len(dsp.istft(S)) == 39936


def test_stft_matches_direct_dft():
    rng = np.random.default_rng(1)
    y = rng.standard_normal(1000)
    S = dsp.stft(y)
    yp = np.pad(y, 128, mode="reflect")
    w = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(256) / 256)
    n = np.arange(256)
    for t in [0, 3, S.shape[1] - 1]:
        fr = yp[128 * t:128 * t + 256] * w
        for k in [0, 1, 17, 64, 128]:
            ref = np.sum(fr * np.exp(-2j * np.pi * n * k / 256))
            assert abs(S[k, t] - ref) < 1e-4 * max(1.0, abs(ref))


def test_stft_parseval_per_frame():
    rng = np.random.default_rng(2)
    y = rng.standard_normal(4096)
    fr = dsp.frame_signal(y) * dsp.hann_periodic()[None]
    S = np.fft.rfft(fr, axis=1)
    e_time = np.sum(fr ** 2, axis=1)
    w = np.ones(129) * 2
    w[0] = w[-1] = 1
    e_freq = np.sum(w * np.abs(S) ** 2, axis=1) / 256
    np.testing.assert_allclose(e_time, e_freq, rtol=1e-10)


@pytest.mark.parametrize("conj", [False, True])
def test_istft_perfect_reconstruction(conj):
    rng = np.random.default_rng(3)
    y = rng.standard_normal(32000)
    r = dsp.istft(dsp.stft(y, conj=conj), conj=conj)
    assert r.shape == (32000,)
    np.testing.assert_allclose(r, y, atol=2e-5)


def test_normalise_and_mix():
    rng = np.random.default_rng(4)
    x = rng.standard_normal(100) + 3.0
    n = dsp.normalise_source(x, 120)
    assert n.shape == (120,) and abs(np.max(np.abs(n[:100])) - 1.0) < 1e-12 and np.all(n[100:] == 0)
    s, m = dsp.mix_sources([n, n], [2.0, 1.0])
    np.testing.assert_allclose(m, 3 * n)


def test_gain_rules_match_synth():
    u = np.array([[0.3, 0.9], [0.7, 0.1]])
    g = synth.gains_for(u, 2)
    assert np.allclose(g[0], dsp.gains_2spk_db(0.3, 0.9)) and np.allclose(g[1], dsp.gains_2spk_db(0.7, 0.1))
    g3 = synth.gains_for(u, 3)
    assert np.allclose(g3[0], dsp.gains_3spk_db(0.3, 0.9))


def test_lstm_cell_equations_match_torch():
    """R9: restate one LSTM step by hand and check torch.nn.LSTM (the oracle's cell)."""
    torch.manual_seed(0)
    rnn = torch.nn.LSTM(5, 4, batch_first=True)
    x = torch.randn(2, 3, 5)
    out, _ = rnn(x)
    W, U, b1, b2 = rnn.weight_ih_l0, rnn.weight_hh_l0, rnn.bias_ih_l0, rnn.bias_hh_l0
    h = torch.zeros(2, 4)
    c = torch.zeros(2, 4)
    for t in range(3):
        g = x[:, t] @ W.T + b1 + h @ U.T + b2
        i, f, gg, o = g.chunk(4, 1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        assert torch.allclose(out[:, t], h, atol=1e-6)


def test_gru_cell_equations_match_torch():
    torch.manual_seed(0)
    rnn = torch.nn.GRU(5, 4, batch_first=True)
    x = torch.randn(2, 3, 5)
    out, _ = rnn(x)
    W, U, b1, b2 = rnn.weight_ih_l0, rnn.weight_hh_l0, rnn.bias_ih_l0, rnn.bias_hh_l0
    h = torch.zeros(2, 4)
    for t in range(3):
        gi = x[:, t] @ W.T + b1
        gh = h @ U.T + b2
        ir, iz, inn = gi.chunk(3, 1)
        hr, hz, hn = gh.chunk(3, 1)
        r, z = torch.sigmoid(ir + hr), torch.sigmoid(iz + hz)
        n = torch.tanh(inn + r * hn)
        h = (1 - z) * n + z * h
        assert torch.allclose(out[:, t], h, atol=1e-6)


def test_pit_reduces_to_label_order_when_identity_is_optimal():
    torch.manual_seed(0)
    B, K, T, F = 3, 2, 5, 7
    X = torch.rand(B, T, F)
    mask = torch.rand(B, K, T, F)
    Y = mask * X[:, None] + 0.01 * torch.rand(B, K, T, F)
    perm, _ = model.pit_assign(mask, X, Y)
    assert perm.tolist() == [[0, 1]] * B
    l_pit, _ = model.loss_pit(mask, X, Y)
    l_lab, _ = model.loss_label_ordered(mask, X, Y)
    assert torch.allclose(l_pit, l_lab)
    # swapped targets -> PIT finds the swap and gives the same loss
    perm2, _ = model.pit_assign(mask, X, Y.flip(1))
    assert perm2.tolist() == [[1, 0]] * B
    assert torch.allclose(model.loss_pit(mask, X, Y.flip(1))[0], l_lab)


def test_mse_gradient_closed_form():
    torch.manual_seed(0)
    B, K, T, F = 2, 2, 3, 4
    X = torch.rand(B, T, F)
    Y = torch.rand(B, K, T, F)
    m = torch.rand(B, K, T, F, requires_grad=True)
    loss, _ = model.loss_label_ordered(m, X, Y)
    loss.backward()
    pred = m.detach() * X[:, None]
    g = 2 * (pred - Y) * X[:, None] / (B * K * T * F) + 0.5 * 2 * (m.detach().sum(1, keepdim=True) - 1) / (B * T * F)
    assert torch.allclose(m.grad, g, atol=1e-7)


def test_top_k_mask_and_label_vector():
    pro = torch.tensor([[0.1, 0.9, 0.6, 0.2], [0.8, 0.1, 0.1, 0.7]])
    m = model.top_k_mask(pro, 0.5, 4)
    assert m.tolist() == [[0, 1, 1, 0], [1, 0, 0, 1]]
    y_spk, y_map = model.multi_label_vector([["b", "c"], ["a", "d"]], {"a": 0, "b": 1, "c": 2, "d": 3})
    assert y_spk == [[1, 2], [0, 3]] and (y_map == m.numpy()).all()


def test_crm_inverse_compression_hazard():
    """cRM numerics: ~20*e for small energies; non-finite past |e| ~ 9.02 in fp32."""
    V = torch.ones(1, 1, 1, 1)
    for e, finite in [(0.5, True), (4.0, True), (9.5, False)]:
        q = torch.tensor([[[e, e]]])
        m = model.attention_crm(V, q)
        assert bool(torch.isfinite(m).all()) == finite
        if e <= 4.0:
            assert abs(float(m[..., 0]) - 20 * e) / (20 * e) < 1e-4


def test_golden_fixture_is_reproduced_by_oracle():
    import os
    from conftest import ROOT
    g = np.load(os.path.join(ROOT, "tests", "golden", "stft_golden.npz"))
    for i in range(g["x"].shape[0]):
        S = dsp.stft_tf(g["x"][i].astype(np.float64))
        np.testing.assert_allclose(S.real, g["re"][i], atol=1e-5)
        np.testing.assert_allclose(S.imag, g["im"][i], atol=1e-5)
        np.testing.assert_allclose(dsp.istft(S.T), g["y_rec"][i], atol=1e-6)


def test_recursive_oracle_selection_known_answers():
    """GRID.py:227-244 top_k_mask with sort_index and the seen-speaker filter (GRID.py:394-399)."""
    from oracle import recursive as orc
    prob = torch.tensor([[0.5, 0.9, 0.9, 0.2, 0.99], [0.1, 0.1, 0.2, 0.05, 0.3]])
    final, sidx, cnt = orc.top_k_sort_index(prob, 0.5, 3)
    assert sidx.tolist() == [[4, 1, 2], [4, 2, 0]]
    assert cnt.tolist() == [3, 0]
    assert final[0].tolist() == [0, 1, 1, 0, 1] and final[1].sum() == 0
    assert orc.choose(sidx, cnt, [[4, 1], []]) == [2, -1]
    assert orc.choose(sidx, cnt, [[4, 1, 2], []]) == [-1, -1]


def test_recursive_oracle_two_steps_tiny():
    """The loop on a tiny constant model: step 1 picks the classifier's top speaker, step 2
    the best unseen one; final masks are computed on the original mixture."""
    from oracle import recursive as orc
    B, T, F, E, N = 1, 3, 4, 2, 5
    emb = torch.randn(N, E, generator=torch.Generator().manual_seed(0))
    V = torch.randn(B, T, F, E, generator=torch.Generator().manual_seed(1))
    probs = [torch.tensor([[0.1, 0.8, 0.3, 0.9, 0.2]]), torch.tensor([[0.1, 0.2, 0.3, 0.95, 0.6]])]
    calls = []

    def cls(x):
        calls.append(x.clone())
        return probs[len(calls) - 1]

    X = torch.rand(B, T, F) + 0.5
    out = orc.recursive_extract(lambda x: (V, None), cls, emb, X)
    assert out["spk"].tolist() == [[3, 4]]
    m1 = torch.sigmoid(torch.einsum("btfe,e->btf", V, emb[3]))[0]
    assert torch.allclose(calls[1][0], (1 - m1) * X[0])
    assert torch.allclose(out["masks"][0, 1], torch.sigmoid(torch.einsum("btfe,e->btf", V, emb[4]))[0])


def test_bss_eval_oracle_known_answers():
    """BSS_EVAL v3 restatement (oracle/bss_eval.py): swapped estimates -> permutation (1, 0);
    an estimate that is a delayed, scaled copy of its source plus another source's leakage
    plus white noise -> SIR / SAR close to the construction's energy ratios; and the
    explicit projection equals a direct least-squares fit on the delay matrix."""
    from oracle import bss_eval as be
    rng = np.random.default_rng(0)
    N, flen = 3000, 32
    s = rng.standard_normal((2, N))
    noise = rng.standard_normal((2, N)) * 0.1
    est = np.stack([0.8 * np.roll(s[1], 3) + 0.05 * s[0] + noise[0], 1.2 * s[0] + 0.1 * s[1] + noise[1]])
    sdr, sir, sar, perm = be.bss_eval_sources(s, est, flen=flen)
    assert perm.tolist() == [1, 0]
    # source 0 <- estimate 1: |s_true|^2 = 1.44 |s0|^2, interference 0.01 |s1|^2, artifacts = noise
    assert abs(sir[0] - 10 * np.log10(1.44 / 0.01)) < 0.5
    assert abs(sar[0] - 10 * np.log10((1.44 + 0.01) / 0.01)) < 0.5
    # explicit projection == direct least squares on the (N + flen - 1) x (2 flen) delay matrix
    A = np.zeros((N + flen - 1, 2 * flen))
    for i in range(2):
        for a in range(flen):
            A[a:a + N, i * flen + a] = s[i]
    e = np.hstack((est[0], np.zeros(flen - 1)))
    c = np.linalg.lstsq(A, e, rcond=None)[0]
    assert np.allclose(A @ c, be._project(s, est[0], flen), atol=1e-8)
