"""Shared batch builder of the compat ``predata_*`` loaders: synthetic sources for the
speakers of a split, the reference's per-source normalisation + gain rules and its
STFT features, computed on the GPU kernels (dl4ss_mix_sources, dl4ss_stft_fwd) and
handed back in the reference's numpy batch-dict layout."""
import random

import numpy as np
import torch

from dl4ss_amd import ops, synth


def draw_shifts(lengths):
    """The list loaders' AUGMENT_DATA draw, one per source in line order:
    ``random_shift = random.sample(range(len(signal)), 1)[0]`` over the cropped source's
    own length (TDAA_beta/predata_fromList.py:150-151, predata_fromList_cRM_123.py:198-200),
    on the module-level ``random`` like the reference.  lengths (B, K) -> (B, K) int32."""
    L = np.asarray(lengths)
    out = np.zeros(L.shape, np.int32)
    for b in range(L.shape[0]):
        for k in range(L.shape[1]):
            out[b, k] = random.sample(range(int(L[b, k])), 1)[0]
    return out


def torch_multi_augment(cfg, n):
    """Torch_multi/predata_multiAims_dB.py:164-166 (and _3dB.py:179-181) with AUGMENT_DATA set:
    the shift is drawn like the list loaders' but applied as ``signal[s:] + signal[:s]``, a
    numpy broadcast of lengths n-s and s that raises for every s outside {1, n-1, n/2}.  The
    reference therefore stops at its first source with this ValueError (with probability
    1 - 3/n; config_WSJ0_dB.py:112 sets the flag, and Torch_multi/ holds no config_WSJ0_dB of
    its own).  This build raises the same error; for the three shifts where numpy broadcasts,
    the reference continues with a folded SUM of two slices (oracle.dsp.augment_torch_multi,
    pinned by tests/golden/ref_r1_augment.npz), which this build does not reproduce -- it
    raises NotImplementedError there instead of training on different data."""
    if not getattr(cfg, "AUGMENT_DATA", False):
        return
    s = random.sample(range(n), 1)[0]
    a, b = n - s, s
    if a == b or a == 1 or b == 1:
        raise NotImplementedError(
            "AUGMENT_DATA with the Torch_multi loaders: the reference's signal[s:] + signal[:s] "
            f"(predata_multiAims_dB.py:166) broadcasts for s={s} of n={n} into a folded sum, not reproduced here")
    raise ValueError(f"operands could not be broadcast together with shapes ({a},) ({b},) ")


def split_speakers(cfg, split):
    """Sorted speaker names of a split (stand-ins for the WSJ0 speaker dirs)."""
    n = {"train": cfg.NUM_SPEAKERS_TRAIN, "valid": cfg.NUM_SPEAKERS_EVAL, "eval": cfg.NUM_SPEAKERS_EVAL,
         "test": cfg.NUM_SPEAKERS_TEST, "eval_test": cfg.NUM_SPEAKERS_TEST}[split]
    prefix = {"train": "s", "valid": "v", "eval": "v", "test": "t", "eval_test": "t"}[split]
    return [f"{prefix}{i:03d}" for i in range(n)]


def gains_of(cfg, u, K, rule):
    """Per-source gains (B, K) of the reference loaders' dB rules:

    * ``"none"``  predata_multiAims.py:177 (the dB branch is ``if 0 and ...``): all 1;
    * ``"db2"``   predata_multiAims_dB.py:124-130: 10^(dB/20 U) on one random channel, only
      when MIN_MIX == MAX_MIX == 2 (else all 1);
    * ``"db3"``   predata_multiAims_3dB.py:124-137,192-217: the 2-channel rule for a 2-speaker
      mixture, and normal / large / small gains 10^(dB/20 0.5), 10^(dB/20 (0.5+0.5U)),
      10^(dB/20 0.5U) for a 3-speaker one when MAX_MIX == 3.
    """
    B = u.shape[0]
    one = np.ones((B, K))
    db = float(getattr(cfg, "dB", 0) or 0)
    if rule == "none" or not db:
        return one
    if rule == "db2":
        return synth.gains_for(u, K, db=db) if (cfg.MIN_MIX == cfg.MAX_MIX == 2 and K == 2) else one
    if rule == "db3":
        if K == 2 or (K == 3 and cfg.MAX_MIX == 3):
            return synth.gains_for(u, K, db=db)
        return one
    raise ValueError(rule)


def list_path(split, k, root="./create-speaker-mixtures/"):
    """predata_fromList.py:80-86: the WSJ0-mix list of a split and mixture size."""
    tag = {"train": "tr", "valid": "cv", "test": "tt"}.get(split)
    return None if tag is None else root + "mix_{}_spk_{}.txt".format(k, tag)


def list_prepare_data(cfg, mode, split, complex_targets, mix_k, seed=1):
    """The list-driven loaders (TDAA_beta/predata_fromList.py:45-236,
    predata_fromList_cRM_123.py:90-293): ``batch_total = lines // BATCH_SIZE`` batches per
    epoch, then ``False`` for every later ``next()`` (:100-102; the drivers break on it).
    With the list file and ``aim_path/data`` wavs present the batches are the real mixtures
    (``dl4ss_amd.wsj0list``: the reference's regexes, per-line dB gains 10^(dB/20)); without
    them (no WSJ0 here) each of LINES_PER_EPOCH synthetic lines draws its dB like the
    wsj0-mix lists (uniform in [-2.5, 2.5])."""
    import os

    from dl4ss_amd import wsj0list

    lp = list_path(split, mix_k)
    data_path = cfg.aim_path + "/data"
    B = cfg.BATCH_SIZE
    # AUGMENT_DATA rotates every TRAIN source (predata_fromList_cRM_123.py:198: `and
    # train_or_test=='train'`); the shifts run through dl4ss_mix_sources_rot on the GPU
    augment = bool(getattr(cfg, "AUGMENT_DATA", False)) and split == "train"
    if lp and os.path.exists(lp) and os.path.isdir(os.path.join(data_path, "train")):
        all_spk = sorted(os.listdir(os.path.join(data_path, "train")))
        lb = wsj0list.ListBatches(lp, data_path, split, B, cfg.MAX_LEN, shuffle=bool(cfg.SHUFFLE_BATCH), seed=seed,
                                  augment=augment)
        batch_total = lb.batch_total
        dev = torch.device("cuda")

        def batches():
            for bt in lb:
                f = wsj0list.features(bt, dev, complex_sources=complex_targets)
                yield dict(src=f["src"], mix=f["mix"], mix_c=f["mix_complex"], mix_mag=f["mix_mag"],
                           src_feat=f["src_spec"], names=bt["speakers"])
    else:
        all_spk = split_speakers(cfg, "train")
        batch_total = LINES_PER_EPOCH.get(split, 3000) // B
        # the cv lines of wsj0-mix use the TRAINING speakers (predata_fromList.py:129-132 reads
        # every split but 'test' from data/train), so the labels stay in the global dict
        maker = BatchMaker(cfg, "test" if split == "test" else "train", mix_k,
                           seed_offset={"train": 0, "valid": 104729}.get(split, 0))
        rng = np.random.default_rng(getattr(cfg, "DATA_SEED", 1) + seed)

        def batches():
            for _ in range(batch_total):
                db = rng.uniform(-2.5, 2.5, size=(B, mix_k))
                yield maker.make(B, complex_targets=complex_targets, db_list=db, augment=augment)
    for dev_batch in batches():
        if mode == "global":
            T, F = dev_batch["mix_mag"].shape[1:3]
            yield (all_spk, {s: i for i, s in enumerate(all_spk)}, {i: s for i, s in enumerate(all_spk)}, T, F, 32,
                   len(all_spk), batch_total)
        elif mode == "once":
            d = to_reference_dict(dev_batch, complex_targets=complex_targets)
            d["num_all_spk"] = len(all_spk)
            d["batch_total"] = batch_total
            yield d
    while True:  # epoch over
        yield False


LINES_PER_EPOCH = {"train": 20000, "valid": 5000, "test": 3000}


class BatchMaker:
    """One generator's state: the synthetic source stream of a split."""

    def __init__(self, cfg, split, k, seed_offset=0):
        self.cfg = cfg
        self.speakers = split_speakers(cfg, split)
        self.k = k
        sd = getattr(cfg, "DATA_SEED", 1) + seed_offset + {"train": 0, "valid": 1, "eval": 1, "test": 2,
                                                            "eval_test": 2}[split] * 7919
        self.gen = synth.SyntheticMixtures(n_samples=cfg.MAX_LEN, k=k, num_labels=len(self.speakers), seed=sd)

    def make(self, B, complex_targets=False, db_list=None, gain_rule="db2", augment=False):
        """Returns the device tensors of one batch: dict with src (B,K,N) scaled sources,
        mix (B,N), mix_c (B,T,F,2), mix_mag (B,T,F), src_feat (B,K,T,F) magnitude or
        (B,K,T,F,2) complex, names (B lists of K names).  gain_rule: see gains_of.
        augment: the list loaders' train-split rotation (draw_shifts); the Torch_multi
        loaders pass ``augment="torch_multi"`` (torch_multi_augment)."""
        cfg = self.cfg
        N, K = cfg.MAX_LEN, self.k
        if augment == "torch_multi":
            torch_multi_augment(cfg, N)
            augment = False
        src, spk, u = self.gen.batch(B)
        if db_list is not None:  # list-driven loaders: gains 10^(dB_i/20) (predata_fromList_cRM_123.py:206,227)
            gains = 10.0 ** (np.asarray(db_list, dtype=np.float64) / 20.0)
        else:
            gains = gains_of(cfg, u, K, gain_rule)
        dev = torch.device("cuda")
        raw = torch.from_numpy(src.astype(np.float32)).to(dev)
        g = torch.from_numpy(np.ascontiguousarray(gains, dtype=np.float32)).to(dev)
        shifts = torch.from_numpy(draw_shifts(np.full((B, K), N))).to(dev) if augment else None
        s, m = ops.mix_sources(raw, g, shifts=shifts)
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
