"""``lrs`` (the reference's remote-logging helper, ``EvalVer.py:22,495-496,560-576``) as a
local sink: ``send(*args)`` appends one JSON line to ``$DL4SS_LRS_LOG`` when it is set and
is a no-op otherwise.  Tensors / numpy scalars are written as floats."""
import json
import os


def _plain(x):
    try:
        import numpy as np
        import torch

        if isinstance(x, torch.Tensor):
            return x.detach().cpu().tolist()
        if isinstance(x, np.generic):
            return x.item()
        if isinstance(x, np.ndarray):
            return x.tolist()
    except ImportError:
        pass
    return x if isinstance(x, (int, float, str, bool, type(None), list, dict)) else str(x)


def send(*args, **kwargs):
    path = os.environ.get("DL4SS_LRS_LOG")
    if not path:
        return
    rec = {"args": [_plain(a) for a in args]}
    if kwargs:
        rec["kwargs"] = {k: _plain(v) for k, v in kwargs.items()}
    with open(path, "a") as f:
        f.write(json.dumps(rec) + "\n")
