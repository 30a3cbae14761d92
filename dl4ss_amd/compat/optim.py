"""``torch.optim.Adam`` stand-in for the driver mirrors: the same constructor (a list of
``{'params': ...}`` groups, ``lr``, ``betas``, ``eps``), ``param_groups`` (so the reference's
LR-halving lines ``for ee in optimizer.param_groups: ee['lr'] /= 2`` work unchanged,
EvalVer.py:570-575), ``zero_grad`` and ``step`` -- with the update on the HIP Adam kernel
(dl4ss_adam: torch's Adam arithmetic, bias corrections in double on the host), one launch
per parameter.  Parameters without a gradient (the discarded classifier, the unused
'align' attention weights) are skipped, as torch skips them.
"""
import torch

from dl4ss_amd import ops


class Adam:
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        groups = list(params)
        if groups and not isinstance(groups[0], dict):
            groups = [{"params": groups}]
        self.param_groups = []
        for g in groups:
            g = dict(g)
            g["params"] = list(g["params"])
            g.setdefault("lr", lr)
            g.setdefault("betas", betas)
            g.setdefault("eps", eps)
            self.param_groups.append(g)
        self.state = {}

    def zero_grad(self):
        for g in self.param_groups:
            for p in g["params"]:
                p.grad = None

    @torch.no_grad()
    def step(self):
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state.get(p)
                if st is None:
                    st = self.state[p] = {"step": 0, "m": torch.zeros_like(p), "v": torch.zeros_like(p)}
                st["step"] += 1
                ops.adam_(p.data, p.grad.contiguous(), st["m"], st["v"], st["step"], g["lr"], g["betas"], g["eps"])
