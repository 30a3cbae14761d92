"""``myNet`` of the reference (Torch_multi/myNet.py), hosting the separation modules.

The reference drivers define MIX_SPEECH / MIX_SPEECH_classifier / SPEECH_EMBEDDING /
ADDJUST / ATTENTION / top_k_mask inside each ``main_run_*.py``; SURVEY section 8b makes
the build's ``myNet`` export them.  Constructor signatures, parameter names (so the
reference ``state_dict`` keys load unchanged) and forward semantics follow:

  MIX_SPEECH             Torch_multi/main_run.py:258-282 (BiGRU, returns V);
                         TDAA_beta/main_run_sstune_EvalVer.py:277-303 (BiLSTM-4L, returns (V, h));
                         main_run_sstune_cRM_EvalVer.py:340-365 (BiGRU, returns (V, h))
  MIX_SPEECH_classifier  main_run.py:284-305, EvalVer.py:305-326
  SPEECH_EMBEDDING       main_run.py:307-327 (dense, masked), EvalVer.py:348-361 (gather),
                         cRM:390-406 (width 2E)
  ADDJUST                EvalVer.py:363-377, cRM:408-426
  ATTENTION              EvalVer.py:199-242 ('dot'), cRM:247-271 (cRM 'dot' branch)
  top_k_mask             main_run.py:340-355, EvalVer.py:390-405

Forward and backward of the recurrence, every Linear / GEMM, the attention, the
gather and top_k_mask run on the HIP kernels (``dl4ss_amd.autograd``); only
reshapes, time means, concatenations and the classifier's sigmoid are torch glue.  The
Inception-v3 video branch (``inception_v3`` / ``Inception3``, ``_inception.py``) is off
the separation path (VIDEO_QUERY is constructed by main_run.py:407 but never called):
it constructs, loads the reference's ImageNet file by name when present, and runs on
plain torch.
"""
import math

import numpy as np
import torch
from torch import nn

from dl4ss_amd import autograd as ag

try:
    from . import config
except ImportError:  # imported by its bare name (compat.install())
    import config

__all__ = ['Inception3', 'inception_v3', 'BiRNN', 'MIX_SPEECH', 'MIX_SPEECH_classifier', 'SPEECH_EMBEDDING',
           'ADDJUST', 'ATTENTION', 'top_k_mask']


try:  # Torch_multi/myNet.py:17-330: the VIDEO_QUERY image net (off the audio path; plain torch)
    from ._inception import Inception3, inception_v3  # noqa: F401
except ImportError:  # imported by its bare name (compat.install())
    from dl4ss_amd.compat._inception import Inception3, inception_v3  # noqa: F401


class BiRNN(nn.Module):
    """Drop-in for nn.LSTM / nn.GRU(input_size, hidden_size, num_layers, batch_first=True,
    bidirectional=True): same parameter names (weight_ih_l{k}[_reverse], ...), torch's
    default init, forward returns (out (B,T,2H), None) -- the reference drivers never
    use the final state (``x, hidden = self.layer(x)``)."""

    def __init__(self, mode, input_size, hidden_size, num_layers=1, batch_first=True, bidirectional=True,
                 precision=None):
        super().__init__()
        if not (batch_first and bidirectional):
            raise ValueError("the HIP recurrence is batch_first and bidirectional (as every reference use)")
        self.mode = mode.lower()
        if self.mode not in ("lstm", "gru"):
            raise ValueError(mode)
        self.input_size, self.hidden_size, self.num_layers = input_size, hidden_size, num_layers
        self.precision = precision
        G = (4 if self.mode == "lstm" else 3) * hidden_size
        for l in range(num_layers):
            d_in = input_size if l == 0 else 2 * hidden_size
            for sfx in ("", "_reverse"):
                setattr(self, f"weight_ih_l{l}{sfx}", nn.Parameter(torch.empty(G, d_in)))
                setattr(self, f"weight_hh_l{l}{sfx}", nn.Parameter(torch.empty(G, hidden_size)))
                setattr(self, f"bias_ih_l{l}{sfx}", nn.Parameter(torch.empty(G)))
                setattr(self, f"bias_hh_l{l}{sfx}", nn.Parameter(torch.empty(G)))
        self.reset_parameters()

    def reset_parameters(self):
        k = 1.0 / math.sqrt(self.hidden_size)  # torch RNN default: U(-1/sqrt(H), 1/sqrt(H))
        for p in self.parameters():
            nn.init.uniform_(p, -k, k)

    def forward(self, x):
        prec = self.precision or getattr(config, "PRECISION", "fp32")
        h = x.float()
        for l in range(self.num_layers):
            g = lambda n: torch.cat([getattr(self, f"{n}_l{l}"), getattr(self, f"{n}_l{l}_reverse")])  # noqa: E731
            h = ag.BiRNNLayerFn.apply(h, g("weight_ih"), g("bias_ih"), g("weight_hh"), g("bias_hh"), self.mode,
                                      self.hidden_size, prec)
        return h, None


class MIX_SPEECH(nn.Module):
    """V = tanh(Linear(BiRNN(x))).view(B, T, F, E).  ``cell`` / ``num_layers`` default to
    the BiGRU-NUM_LAYERS of Torch_multi/main_run.py; ``return_hidden`` gives the
    (V, h) of the TDAA_beta drivers (EvalVer.py:302, cRM:364)."""

    def __init__(self, input_fre, mix_speech_len, cell=None, num_layers=None, return_hidden=False, precision=None):
        super().__init__()
        self.input_fre, self.mix_speech_len = input_fre, mix_speech_len
        self.return_hidden = return_hidden
        self.precision = precision
        self.layer = BiRNN(cell or getattr(config, "MIX_CELL", "gru"), input_fre, config.HIDDEN_UNITS,
                           num_layers or config.NUM_LAYERS, precision=precision)
        self.Linear = nn.Linear(2 * config.HIDDEN_UNITS, input_fre * config.EMBEDDING_SIZE)

    def forward(self, x):
        h, _ = self.layer(x)
        B, T, D = h.shape
        prec = self.precision or getattr(config, "PRECISION", "fp32")
        v = ag.LinearTanhFn.apply(h.reshape(B * T, D), self.Linear.weight, self.Linear.bias, prec)
        v = v.view(B, T, self.input_fre, -1)
        return (v, h) if self.return_hidden else v


class MIX_SPEECH_classifier(nn.Module):
    """Speaker classifier: sigmoid(Linear(mean_t BiLSTM(x))) (main_run.py:284-305:
    H = HIDDEN_UNITS, NUM_LAYERS; EvalVer.py:305-326: H = 2 HIDDEN_UNITS, 3 layers)."""

    def __init__(self, input_fre, mix_speech_len, num_labels, hidden=None, num_layers=None, precision=None):
        super().__init__()
        self.input_fre, self.mix_speech_len = input_fre, mix_speech_len
        H = hidden or config.HIDDEN_UNITS
        self.layer = BiRNN("lstm", input_fre, H, num_layers or config.NUM_LAYERS, precision=precision)
        self.Linear = nn.Linear(2 * H, num_labels)

    def forward(self, x):
        h, _ = self.layer(x)
        prec = self.layer.precision or getattr(config, "PRECISION", "fp32")
        return torch.sigmoid(ag.LinearFn.apply(torch.mean(h, 1), self.Linear.weight, self.Linear.bias, prec))


class SPEECH_EMBEDDING(nn.Module):
    """forward(input, mask_idx): gather of the selected speakers' rows (B, K, W)
    (EvalVer.py:355-360); forward(input) with a (B, N_lab) 0/1 mask: the dense
    masked form of main_run.py:318-327 (B, N_lab, W), inactive rows 0."""

    def __init__(self, num_labels, embedding_size, max_num_channel, crm=None):
        super().__init__()
        self.num_all, self.max_num_out = num_labels, max_num_channel
        crm = getattr(config, "is_ComlexMask", False) if crm is None else crm
        self.emb_size = 2 * embedding_size if crm else embedding_size
        self.layer = nn.Embedding(num_labels, self.emb_size)

    def forward(self, input, mask_idx=None):
        dev = self.layer.weight.device
        if mask_idx is not None:
            idx = torch.as_tensor(np.array(mask_idx), dtype=torch.int32, device=dev)
            return ag.EmbeddingGatherFn.apply(self.layer.weight, idx)
        m = torch.as_tensor(input, dtype=torch.float32, device=dev)
        B = m.shape[0]
        idx = torch.arange(self.num_all, dtype=torch.int32, device=dev).expand(B, self.num_all).contiguous()
        return ag.EmbeddingGatherFn.apply(self.layer.weight, idx) * m[:, :, None]


class ADDJUST(nn.Module):
    """W [mean_t h ; q] (no bias), shape (B, K, W) (EvalVer.py:363-377); the driver adds q."""

    def __init__(self, hidden_units, embedding_size, crm=None):
        super().__init__()
        crm = getattr(config, "is_ComlexMask", False) if crm is None else crm
        self.hidden_units = hidden_units
        self.emb_size = 2 * embedding_size if crm else embedding_size
        self.layer = nn.Linear(hidden_units + self.emb_size, self.emb_size, bias=False)

    def forward(self, input_hidden, prob_emb):
        B, K = prob_emb.shape[:2]
        x = torch.mean(input_hidden, 1).view(B, 1, self.hidden_units).expand(B, K, self.hidden_units)
        can = torch.cat([x, prob_emb.float()], dim=2).reshape(B * K, -1)
        prec = getattr(config, "PRECISION", "fp32")
        return ag.LinearFn.apply(can, self.layer.weight, None, prec).view(B, K, -1)


class ATTENTION(nn.Module):
    """'dot' mode on the HIP kernel: mask = sigmoid(V . q) (EvalVer.py:216-226); with
    config.is_ComlexMask the cRM branch 10 tanh(V . q_half), (B', T, F, 2) (cRM:259-271).
    'align' keeps its parameters (state_dict compatibility) but is never executed by the
    reference and raises."""

    def __init__(self, hidden_size, mode='dot', crm=None):
        super().__init__()
        self.hidden_size = self.align_hidden_size = hidden_size
        self.mode = mode
        self.crm = getattr(config, "is_ComlexMask", False) if crm is None else crm
        self.Linear_1 = nn.Linear(hidden_size, hidden_size, bias=False)
        self.Linear_2 = nn.Linear(hidden_size, hidden_size, bias=False)
        self.Linear_3 = nn.Linear(hidden_size, 1, bias=False)

    def forward(self, mix_hidden, query):
        if self.mode != 'dot':
            raise NotImplementedError("ATTENTION 'align' is constructed but never run by the reference")
        B = mix_hidden.shape[0]
        shp = mix_hidden.shape
        V = mix_hidden.reshape(B, -1, self.hidden_size)
        q = query.reshape(B, -1)
        mask = ag.AttentionDotFn.apply(V, q, self.crm)
        return mask.view(B, shp[1], shp[2], 2) if self.crm else mask.view(B, shp[1], shp[2])


def top_k_mask(batch_pro, alpha, top_k):
    """main_run.py:340-355: a (B, N) 0/1 float mask of the (at most top_k) entries above
    alpha, computed on the GPU (no sort, no per-row host loop); returned on the CPU as
    the reference's ``final`` tensor.  Ties are broken by the lower index."""
    p = torch.as_tensor(batch_pro, dtype=torch.float32)
    if not p.is_cuda:
        p = p.cuda()
    mask, _, _ = ag.top_k_mask_device(p.detach(), alpha, top_k)
    return mask.cpu()
