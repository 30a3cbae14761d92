"""Why the all-bf16 operand mode misses the north-star 1e-3 on the BiGRU nets (C1 / C3 / C4) and
the mixed mode (exact GEMMs, bf16 recurrent matvec) meets it -- reproduced on CPU by emulation
(tools/bf16_budget.py: the C4 model in fp64 with bf16 rounding inserted where the HIP bf16 step
rounds), so the gap the strict-xfail GPU test records is measured here rather than absorbed by a
looser tolerance.  Reduced size (B = 2, N = 8000) to keep the CPU suite fast; the
full-size numbers are in profiles/r04_parity_configs.jsonl."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import bf16_budget as bb  # noqa: E402

from oracle import model as om  # noqa: E402
from dl4ss_amd import synth  # noqa: E402
from test_step_gpu import _oracle_features  # noqa: E402


def test_bf16_operand_rounding_budget_c4():
    torch.manual_seed(3)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    ref = om.SepModel(cell="gru", num_layers=2, adjust=False)
    sd = {k: v.detach() for k, v in ref.state_dict().items()}
    B, K, N = 2, 3, 8000
    src, spk, u = synth.SyntheticMixtures(n_samples=N, k=K, seed=3).batch(B)
    feats, X, Y = _oracle_features(src, synth.gains_for(u, K), False)
    run = lambda R: bb.forward(sd, "gru", 2, feats, spk, False, R) * X.double()[:, None]  # noqa: E731
    truth = run(set())
    rel = lambda R: float((run(R) - truth).norm() / truth.norm())  # noqa: E731
    every = rel({"feat", "wih", "xin", "rec", "lin", "V"})  # the all-bf16 step's roundings
    mixed = rel({"xin", "rec"})  # bf16 recurrence: h_{t-1}, W_hh and the bf16 layer hand-over
    assert every > 1e-3, every
    assert mixed < 0.6e-3, mixed
    assert every > 2.5 * mixed, (every, mixed)
