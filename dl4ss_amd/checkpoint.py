"""Checkpoint compatibility with the reference's per-module ``params/param_*`` files
(SURVEY section 8f row f4).

The reference saves one ``state_dict`` per module every 5 epochs
(``TDAA_beta/main_run_sstune_EvalVer.py:677-690``: ``..._hidden3d_{epoch}`` = MIX_SPEECH,
``_emblayer_`` = SPEECH_EMBEDDING, ``_adjlayer_`` = ADDJUST, ``_attlayer_`` = ATTENTION,
``_dislayer_`` = Discriminator) and loads them back the same way (``EvalVer.py:545-554``;
the classifier file drops its ``cnn`` keys, ``:547-549``).  Key names inside each file are
the module's own: ``layer.weight_ih_l0[_reverse]`` / ``Linear.weight`` (MIX_SPEECH),
``layer.weight`` (embedding, ADDJUST), ``Linear_{1,2,3}.weight`` (attention).

Files are read with ``torch.load(..., weights_only=True)`` only (no arbitrary unpickling):
torch-0.3 / Python-2 files in the legacy (non-zip) format -- protocol-2 pickles of an
``OrderedDict`` of ``torch._utils._rebuild_tensor`` tensors over ``torch.cuda.FloatStorage``
persistent ids saved on ``cuda:N`` (fixture: ``tests/golden/legacy_py2_torch03``, built
opcode by opcode by ``tests/golden/make_legacy_ckpt.py``) -- load through the same safe
path; a file the safe loader refuses raises.  The flat parameter buffers of ``SepNet`` /
``ClassifierNet`` carry the same names under a module prefix (``mix.``, ``emb.``, ``adj.``),
so loading is a rename and a copy; ``save_reference_params`` writes the reference layout
back (one file per module, legacy-compatible keys).
"""
import os

import torch

PREFIX = {"hidden3d": "mix.", "emblayer": "emb.", "adjlayer": "adj."}


def load_state(path):
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(sd, dict):
        raise ValueError(f"{path}: not a state_dict")
    return {k: (v.data if hasattr(v, "data") else v) for k, v in sd.items()}


def load_reference_params(net, hidden3d=None, emblayer=None, adjlayer=None, strict=True):
    """Load the reference's per-module files into a SepNet (in place).  Missing module files
    are skipped; with ``strict`` every key of a given file must map onto the net AND every
    parameter of the net under that file's module prefix must be in the file (torch's
    ``load_state_dict(strict=True)`` in both directions: a 2-layer hidden3d file does not
    silently leave layers 2-3 of a 4-layer net at their random init)."""
    for kind, path in (("hidden3d", hidden3d), ("emblayer", emblayer), ("adjlayer", adjlayer)):
        if path is None:
            continue
        sd = load_state(path)
        if strict:
            want = {name[len(PREFIX[kind]):] for name, _ in net.specs if name.startswith(PREFIX[kind])}
            missing = sorted(want - set(sd))
            if missing:
                raise KeyError(f"{path}: missing {missing} for this net")
        for k, v in sd.items():
            name = PREFIX[kind] + k
            if name not in net.offsets:
                if strict:
                    raise KeyError(f"{path}: key {k!r} has no counterpart ({name}) in this net")
                continue
            dst = net.view(name)
            if tuple(dst.shape) != tuple(v.shape):
                raise ValueError(f"{path}: {k} has shape {tuple(v.shape)}, the net expects {tuple(dst.shape)}")
            dst.copy_(v.to(torch.float32))
    return net


def load_reference_classifier(cnet, path, strict=True):
    """MIX_SPEECH_classifier file into a ClassifierNet (the ``cnn`` keys dropped, EvalVer.py:547-549)."""
    sd = {k: v for k, v in load_state(path).items() if "cnn" not in k}
    if strict:
        missing = sorted({name for name, _ in cnet.specs} - set(sd))
        if missing:
            raise KeyError(f"{path}: missing {missing} for this classifier")
    for k, v in sd.items():
        if k not in cnet.offsets:
            if strict:
                raise KeyError(f"{path}: key {k!r} has no counterpart in the classifier")
            continue
        dst = cnet.view(k)
        if tuple(dst.shape) != tuple(v.shape):
            raise ValueError(f"{path}: {k} has shape {tuple(v.shape)}, the classifier expects {tuple(dst.shape)}")
        dst.copy_(v.to(torch.float32))
    return cnet


def save_reference_params(net, directory, tag, epoch):
    """Write the reference's file layout ``param_{tag}_{hidden3d,emblayer,adjlayer}_{epoch}``."""
    os.makedirs(directory, exist_ok=True)
    paths = {}
    for kind, pre in PREFIX.items():
        sd = {name[len(pre):]: net.view(name).detach().cpu().clone() for name, _ in net.specs if name.startswith(pre)}
        if not sd:
            continue
        p = os.path.join(directory, f"param_{tag}_{kind}_{epoch}")
        torch.save(sd, p)
        paths[kind] = p
    return paths
