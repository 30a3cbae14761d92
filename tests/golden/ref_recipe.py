"""Shared recipe for the reference-generated step fixtures (TEST INFRASTRUCTURE ONLY).

The fixtures in ``tests/golden/ref_*.npz`` are produced by ``make_ref_fixtures.py``,
which runs the reference's own (py2 -> py3 translated) modules and training-loop
lines in the build container.  Full BiLSTM-4L weights (11.4 M floats) are too large
to commit, so both sides derive the initial weights from this numpy recipe (PCG64
seeded per parameter name: bitwise identical on every machine), and the fixtures
store full small tensors plus fixed random subsets of the large ones.

Names use the build's state-dict prefixes: ``mix.`` (MIX_SPEECH), ``emb.``
(SPEECH_EMBEDDING), ``adj.`` (ADDJUST), ``cls.`` (MIX_SPEECH_classifier).
"""
import os
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SUBSET = 2048  # entries kept per large tensor (indices re-derived from the name, not stored)
FULL_MAX = 65536  # tensors up to this many elements are stored whole


def _rng(seed, name):
    return np.random.Generator(np.random.PCG64([seed, zlib.crc32(name.encode())]))


def init_param(name, shape, hidden, seed):
    """torch's default initialisers restated (nn.LSTM/GRU U(+-1/sqrt(H)), nn.Linear
    U(+-1/sqrt(fan_in)), nn.Embedding N(0, 1)) with a per-name numpy stream."""
    r = _rng(seed, name)
    if name.endswith("emb.layer.weight"):
        return r.standard_normal(shape).astype(np.float32)
    if "_ih_l" in name or "_hh_l" in name:
        k = 1.0 / np.sqrt(hidden)
    elif name.endswith(".bias"):  # MIX_SPEECH.Linear (2H -> F*E) / classifier Linear (2H_cls -> labels)
        k = 1.0 / np.sqrt(2 * hidden)
    else:
        k = 1.0 / np.sqrt(shape[1])
    return r.uniform(-k, k, size=shape).astype(np.float32)


def weights(specs, hidden, seed, cls_hidden=None):
    """specs: [(name, shape)] -> {name: float32 array}."""
    out = {}
    for name, shape in specs:
        h = cls_hidden if name.startswith("cls.") else hidden
        out[name] = init_param(name, tuple(shape), h, seed)
    return out


def subset_index(name, numel, seed=0):
    """Fixed subset of a large tensor's flat indices (sorted)."""
    if numel <= FULL_MAX:
        return None
    r = _rng(seed + 7, name)
    return np.sort(r.choice(numel, size=SUBSET, replace=False)).astype(np.int64)


def pack(prefix, name, arr, out, seed=0):
    """Store arr whole or as (subset indices, values, L2 norm, sum)."""
    a = np.asarray(arr, dtype=np.float32)
    idx = subset_index(name, a.size, seed)
    out[f"{prefix}/{name}/shape"] = np.array(a.shape, dtype=np.int64)
    out[f"{prefix}/{name}/norm"] = np.float64(np.linalg.norm(a.astype(np.float64)))
    out[f"{prefix}/{name}/sum"] = np.float64(a.astype(np.float64).sum())
    if idx is None:
        out[f"{prefix}/{name}/full"] = a
    else:
        out[f"{prefix}/{name}/val"] = a.reshape(-1)[idx]


def stored(fx, prefix, name):
    """The stored entries (whole tensor or its subset) as float64, and the subset (or None)."""
    if f"{prefix}/{name}/full" in fx.files:
        return fx[f"{prefix}/{name}/full"].astype(np.float64).reshape(-1), None
    shape = tuple(fx[f"{prefix}/{name}/shape"])
    return fx[f"{prefix}/{name}/val"].astype(np.float64), subset_index(name, int(np.prod(shape)))


def unpack_names(fx, prefix):
    names = set()
    for k in fx.files:
        if k.startswith(prefix + "/"):
            names.add(k[len(prefix) + 1:].rsplit("/", 1)[0])
    return sorted(names)


def compare(fx, prefix, name, ours):
    """Max abs error of ours over the stored entries, relative to the stored entries'
    max |.|, plus the L2-norm ratio; returns (err, norm_ratio)."""
    ours = np.asarray(ours, dtype=np.float64).reshape(-1)
    if f"{prefix}/{name}/full" in fx.files:
        ref = fx[f"{prefix}/{name}/full"].astype(np.float64).reshape(-1)
        mine = ours
    else:
        ref = fx[f"{prefix}/{name}/val"].astype(np.float64)
        mine = ours[subset_index(name, ours.size)]
    denom = max(np.abs(ref).max(), 1e-30)
    err = float(np.abs(mine - ref).max() / denom)
    nref = float(fx[f"{prefix}/{name}/norm"])
    ratio = float(np.linalg.norm(ours) / nref) if nref > 0 else 1.0
    return err, ratio


def load(name):
    return np.load(os.path.join(HERE, name), allow_pickle=False)


def fixture_weights(fx, specs):
    """The initial weights a fixture was generated with, for the given [(name, shape)]."""
    seed = int(fx["meta/wseed"])
    cls_hidden = int(fx["meta/cls_hidden"]) if "meta/cls_hidden" in fx.files else None
    w = weights(specs, hidden=300, seed=seed, cls_hidden=cls_hidden)
    if "meta/emb_scale" in fx.files and "emb.layer.weight" in w:
        w["emb.layer.weight"] *= np.float32(fx["meta/emb_scale"])
    return w


def check_params(fx, prefix, get, grad_tol, skip=()):
    """Compare every stored tensor under prefix with get(name) -> array; returns {name: err}
    of the failures (max abs error over the stored entries / their max |.| > grad_tol, or an
    L2-norm ratio off by more than grad_tol)."""
    bad = {}
    for name in unpack_names(fx, prefix):
        if name in skip:
            continue
        err, ratio = compare(fx, prefix, name, get(name))
        if err > grad_tol or abs(ratio - 1.0) > grad_tol:
            bad[name] = (err, ratio)
    return bad


def check_adam(fx, get, lr=2e-4):
    """Adam-updated parameters: a first step moves each weight by ~lr*sign(g); a sign
    disagreement is allowed only on a small fraction of entries (gradients at rounding
    level).  Returns {name: (max diff, fraction off)} of the failures."""
    bad = {}
    for name in unpack_names(fx, "param"):
        ref, idx = stored(fx, "param", name)
        ours = np.asarray(get(name), np.float64).reshape(-1)
        if idx is not None:
            ours = ours[idx]
        d = np.abs(ours - ref)
        frac = float((d > 1e-6).mean())
        if d.max() > 2.1 * lr or frac > 2e-3:
            bad[name] = (float(d.max()), frac)
    return bad
