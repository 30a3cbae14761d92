"""Edge cases of the HIP path (empty / ragged / degenerate inputs), each against the CPU
oracle or the defined behaviour: no kernel may fault, hang or return NaN where the
reference's arithmetic is finite."""
import numpy as np
import pytest
import torch

from dl4ss_amd import _lib, ops, synth
from oracle import dsp
from oracle import model as om

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def test_empty_batches_are_noops(dev):
    x = torch.empty(0, 4000, device=dev)
    X, M = ops.stft(x)
    assert X.shape == (0, ops.n_frames(4000), 129, 2) and M.shape[0] == 0
    src = torch.empty(0, 2, 4000, device=dev)
    s, m = ops.mix_sources(src, torch.empty(0, 2, device=dev))
    assert s.numel() == 0 and m.numel() == 0
    torch.cuda.synchronize()


@pytest.mark.parametrize("N", [129, 130, 255, 256, 257, 383])
def test_stft_shortest_signals(dev, N):
    """the shortest signals the boundary accepts (N > n_fft / 2: reflect padding needs no second
    reflection), against librosa's stft restated; T = 1 + N // 128 frames."""
    x = np.random.default_rng(N).standard_normal((3, N)).astype(np.float32)
    X, M = ops.stft(torch.from_numpy(x).to(dev))
    torch.cuda.synchronize()
    assert X.shape[1] == 1 + N // 128
    for i in range(3):
        ref = dsp.stft_tf(x[i])
        assert np.abs(M[i].cpu().numpy() - np.abs(ref)).max() < 1e-4 * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("N", [1, 64, 128])
def test_stft_rejects_signals_within_half_a_frame(dev, N):
    """N <= 128 would need numpy's repeated reflection; the boundary refuses it loudly."""
    with pytest.raises(RuntimeError, match="invalid argument"):
        ops.stft(torch.zeros(2, N, device=dev))


def test_mix_sources_silent_and_ragged_sources(dev):
    """a silent source (peak 0: the reference would divide by zero) becomes zeros, not NaN;
    ragged lengths (list-file wavs) normalise over their own length and zero-pad."""
    N = 5000
    rng = np.random.default_rng(1)
    raw = rng.standard_normal((2, 2, N)).astype(np.float32)
    raw[0, 1] = 0.25  # constant -> zero after mean removal
    lens = np.array([[N, 3000], [17, 4999]], dtype=np.int32)
    gains = np.array([[1.0, 2.0], [0.5, 1.5]], dtype=np.float32)
    s, m = ops.mix_sources(torch.from_numpy(raw).to(dev), torch.from_numpy(gains).to(dev),
                           lengths=torch.from_numpy(lens).to(dev))
    s = s.cpu().numpy()
    assert np.isfinite(s).all() and not s[0, 1].any()
    for b, k in ((0, 0), (1, 0), (1, 1)):
        ref = dsp.normalise_source(raw[b, k, :lens[b, k]].astype(np.float64), N) * gains[b, k]
        assert np.abs(s[b, k] - ref).max() < 1e-5


def test_pit_ties_pick_the_lowest_permutation(dev):
    """identical targets for both channels: every permutation costs the same -> identity (index 0),
    the oracle's rule (om.pit_assign)."""
    from dl4ss_amd import engine
    B, K, N = 2, 2, 3000
    net = engine.SepNet(cell="gru", num_layers=1, device=dev, seed=4)
    tr = engine.SepTrainer(net, B, K, N, mode="pit")
    gen = synth.SyntheticMixtures(n_samples=N, k=K, seed=4)
    src, spk, u = gen.batch(B)
    src[:, 1] = src[:, 0]  # two identical sources -> identical targets
    tr.spk.copy_(torch.from_numpy(spk.astype(np.int32)).to(dev))
    tr.features(torch.from_numpy(src.astype(np.float32)).to(dev), torch.ones(B, K, device=dev))
    tr.forward()
    loss = tr.loss_and_grad()
    torch.cuda.synchronize()
    assert tr.perm.cpu().tolist() == [[0, 1], [0, 1]]
    assert torch.isfinite(loss).all()


def test_top_k_mask_all_below_alpha_and_ties(dev):
    p = torch.tensor([[0.1, 0.2, 0.3], [0.7, 0.7, 0.7]], device=dev)
    mask = torch.empty(2, 3, device=dev)
    idx = torch.empty(2, 2, dtype=torch.int32, device=dev)
    cnt = torch.empty(2, dtype=torch.int32, device=dev)
    _lib.call("dl4ss_top_k_mask", _lib.ptr(p), 2, 3, 0.5, 2, _lib.ptr(mask), _lib.ptr(idx), _lib.ptr(cnt),
              _lib.stream_ptr())
    torch.cuda.synchronize()
    assert mask.cpu().tolist() == [[0, 0, 0], [1, 1, 0]]
    assert idx.cpu().tolist() == [[-1, -1], [0, 1]] and cnt.cpu().tolist() == [0, 2]
    assert torch.equal(mask.cpu(), om.top_k_mask(p.cpu(), 0.5, 2))
