"""Shared batch builder of the compat ``predata_*`` loaders: synthetic sources for the
speakers of a split, the reference's per-source normalisation + gain rules and its
STFT features, computed on the GPU kernels (dl4ss_mix_sources, dl4ss_stft_fwd) and
handed back in the reference's numpy batch-dict layout."""
import numpy as np
import torch

from dl4ss_amd import ops, synth


def split_speakers(cfg, split):
    """Sorted speaker names of a split (stand-ins for the WSJ0 speaker dirs)."""
    n = {"train": cfg.NUM_SPEAKERS_TRAIN, "valid": cfg.NUM_SPEAKERS_EVAL, "eval": cfg.NUM_SPEAKERS_EVAL,
         "test": cfg.NUM_SPEAKERS_TEST, "eval_test": cfg.NUM_SPEAKERS_TEST}[split]
    prefix = {"train": "s", "valid": "v", "eval": "v", "test": "t", "eval_test": "t"}[split]
    return [f"{prefix}{i:03d}" for i in range(n)]


class BatchMaker:
    """One generator's state: the synthetic source stream of a split."""

    def __init__(self, cfg, split, k, seed_offset=0):
        self.cfg = cfg
        self.speakers = split_speakers(cfg, split)
        self.k = k
        sd = getattr(cfg, "DATA_SEED", 1) + seed_offset + {"train": 0, "valid": 1, "eval": 1, "test": 2,
                                                            "eval_test": 2}[split] * 7919
        self.gen = synth.SyntheticMixtures(n_samples=cfg.MAX_LEN, k=k, num_labels=len(self.speakers), seed=sd)

    def make(self, B, complex_targets=False, db_list=None):
        """Returns the device tensors of one batch: dict with src (B,K,N) scaled sources,
        mix (B,N), mix_c (B,T,F,2), mix_mag (B,T,F), src_feat (B,K,T,F) magnitude or
        (B,K,T,F,2) complex, names (B lists of K names)."""
        cfg = self.cfg
        N, K = cfg.MAX_LEN, self.k
        src, spk, u = self.gen.batch(B)
        if db_list is not None:  # list-driven loaders: gains 10^(dB_i/20) (predata_fromList_cRM_123.py:206,227)
            gains = 10.0 ** (np.asarray(db_list, dtype=np.float64) / 20.0)
        else:
            gains = synth.gains_for(u, K, db=float(cfg.dB))
        dev = torch.device("cuda")
        raw = torch.from_numpy(src.astype(np.float32)).to(dev)
        g = torch.from_numpy(np.ascontiguousarray(gains, dtype=np.float32)).to(dev)
        s, m = ops.mix_sources(raw, g)
        Xc, Xm = ops.stft(m, complex_out=True, mag_out=True, log=bool(cfg.IS_LOG_SPECTRAL))
        if complex_targets:
            Sc, _ = ops.stft(s.view(B * K, N), complex_out=True, mag_out=False)
            feat = Sc.view(B, K, *Sc.shape[1:])
        else:
            _, Sm = ops.stft(s.view(B * K, N), complex_out=False, mag_out=True)
            feat = Sm.view(B, K, *Sm.shape[1:])
        names = [[self.speakers[i] for i in row] for row in spk]
        return dict(src=s, mix=m, mix_c=Xc, mix_mag=Xm, src_feat=feat, names=names)


def to_reference_dict(t, complex_targets=False):
    """Device batch -> the reference's numpy batch dict (float64 waves, float32
    features, complex64 mix_phase)."""
    src = t["src"].double().cpu().numpy()
    mix = t["mix"].double().cpu().numpy()
    mix_c = t["mix_c"].cpu().numpy()
    feat = t["src_feat"].cpu().numpy()
    names = t["names"]
    d = {
        "mix_wav": mix,
        "mix_feas": t["mix_mag"].cpu().numpy(),
        "mix_phase": (mix_c[..., 0] + 1j * mix_c[..., 1]).astype(np.complex64),
        "aim_fea": np.stack([feat[b, 0] for b in range(len(names))]),
        "aim_spkname": [row[0] for row in names],
        "query": np.array([]),
        "multi_spk_fea_list": [{n: feat[b, k] for k, n in enumerate(row)} for b, row in enumerate(names)],
        "multi_spk_wav_list": [{n: src[b, k] for k, n in enumerate(row)} for b, row in enumerate(names)],
    }
    if complex_targets:
        d["mix_mag"] = mix_c
    return d
