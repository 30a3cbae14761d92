"""The hot-path kernels as ``torch.library`` custom ops (namespace ``dl4ss``), SURVEY §8(b):
"Python registers these as torch.library custom ops with autograd.Function backward".

Each op is a schema'd PyTorch operator over one or a few C-ABI calls of
``libdl4ss_hip.so`` (``include/dl4ss_hip.h``), with

* a CUDA implementation only -- a CPU tensor raises (there is no CPU fallback; the CPU
  restatement in ``oracle/`` is test infrastructure, never called from here);
* a fake (meta) implementation, so shapes propagate under ``FakeTensorMode`` / meta tensors
  and the ops trace into ``torch.compile`` / ``torch.export`` graphs as single nodes;
* ``register_autograd`` backwards for the differentiable ones, whose gradients are
  themselves ``dl4ss::*_bwd`` ops.

Ops (reference call sites they replace):

=====================================  ==========================================================
``dl4ss::stft_mag(x, log)``            |STFT| / log|STFT| features (predata_multiAims_dB.py:199-203)
``dl4ss::stft_complex(x, conj)``       complex STFT [re, im] (predata_fromList_cRM_123.py:224-229)
``dl4ss::istft(S, conj)``              librosa istft (EvalVer.py:64-65, cRM_EvalVer.py:98-99)
``dl4ss::istft_apply(X, aux, k, crm,   mask / cRM apply + iSTFT (EvalVer.py:56-65,
conj)``                                cRM_EvalVer.py:96-99,720-728)
``dl4ss::mix_sources(raw, gains)``     normalise + gain + sum (predata_multiAims_dB.py:156-197)
``dl4ss::birnn_layer(x, w_ih, b_ih,    one bidirectional LSTM / GRU layer (EvalVer.py:282-293,
w_hh, b_hh, cell, H, precision)``      main_run.py:263-273); returns (out, hprev, act, cs)
``dl4ss::linear_tanh(x, w, b, prec)``  MIX_SPEECH head tanh(Linear) (EvalVer.py:290,298-299)
``dl4ss::attention_dot(V, q, crm)``    ATTENTION 'dot' mask (EvalVer.py:216-226, cRM:259-271)
``dl4ss::top_k_mask(p, alpha, k)``     top_k_mask (EvalVer.py:390-405)
=====================================  ==========================================================

``birnn_layer`` returns its saved activations as extra outputs (a custom op cannot stash
tensors); ``birnn(x, ...)`` below returns the layer output only.
"""
from typing import Tuple

import torch
from torch import Tensor

# every op computes and returns fp32 (the real ops reject other dtypes): the fake kernels say so
F32 = dict(dtype=torch.float32)

from . import _lib, autograd as ag, ops

NS = "dl4ss"
_CUDA = ("cuda",)


def _op(name):
    return torch.library.custom_op(f"{NS}::{name}", mutates_args=(), device_types=_CUDA)


# --------------------------------------------------------------------------- STFT / iSTFT / mixing
@_op("stft_mag")
def stft_mag(x: Tensor, log: bool = False) -> Tensor:
    return ops.stft(ag._c(x), complex_out=False, mag_out=True, log=log)[1]


@stft_mag.register_fake
def _(x, log=False):
    N = x.shape[-1]
    return x.new_empty(*x.shape[:-1], ops.n_frames(N), ops.F_BINS, **F32)


@_op("stft_complex")
def stft_complex(x: Tensor, conj: bool = False) -> Tensor:
    return ops.stft(ag._c(x), complex_out=True, mag_out=False, conj=conj)[0]


@stft_complex.register_fake
def _(x, conj=False):
    N = x.shape[-1]
    return x.new_empty(*x.shape[:-1], ops.n_frames(N), ops.F_BINS, 2, **F32)


@_op("istft")
def istft(S: Tensor, conj: bool = False) -> Tensor:
    return ops.istft(ag._c(S), conj=conj)


@istft.register_fake
def _(S, conj=False):
    return S.new_empty(*S.shape[:-3], ops.HOP * (S.shape[-3] - 1), **F32)


@_op("istft_apply")
def istft_apply(X: Tensor, aux: Tensor, k_per_mix: int, crm: bool, conj: bool = False) -> Tensor:
    """X (B, T, 129, 2) mixture spectra; aux (B*k, T, 129) masked magnitudes (crm False) or
    (B*k, T, 129, 2) complex ratio masks (crm True) -> (B*k, 128 (T - 1)) waveforms."""
    X, aux = ag._c(X), ag._c(aux)
    T = X.shape[-3]
    n_sig = aux.shape[0]
    if X.shape[0] * k_per_mix != n_sig:
        raise RuntimeError("istft_apply: aux rows must be k_per_mix per mixture")
    y = torch.empty(n_sig, ops.HOP * (T - 1), device=X.device)
    _lib.call("dl4ss_istft_apply", _lib.ptr(X), _lib.ptr(aux), n_sig, k_per_mix, T, 1 if crm else 0, int(conj),
              _lib.ptr(y), _lib.stream_ptr())
    return y


@istft_apply.register_fake
def _(X, aux, k_per_mix, crm, conj=False):
    return X.new_empty(aux.shape[0], ops.HOP * (X.shape[-3] - 1), **F32)


@_op("mix_sources")
def mix_sources(raw: Tensor, gains: Tensor) -> Tuple[Tensor, Tensor]:
    return ops.mix_sources(ag._c(raw), ag._c(gains))


@mix_sources.register_fake
def _(raw, gains):
    B, K, N = raw.shape
    return raw.new_empty(B, K, N, **F32), raw.new_empty(B, N, **F32)


# --------------------------------------------------------------------------- BiRNN layer
@_op("birnn_layer")
def birnn_layer(x: Tensor, w_ih: Tensor, b_ih: Tensor, w_hh: Tensor, b_hh: Tensor, cell: str, H: int,
                precision: str) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    out, hprev, act, cs = ag.birnn_fwd_impl(x, w_ih, b_ih, w_hh, b_hh, cell, H, precision)
    return out, hprev, act, cs if cs is not None else x.new_empty(0)


@birnn_layer.register_fake
def _(x, w_ih, b_ih, w_hh, b_hh, cell, H, precision):
    B, T, _ = x.shape
    cs = x.new_empty(B, T, 2, H, **F32) if cell == "lstm" else x.new_empty(0, **F32)
    return (x.new_empty(B, T, 2 * H, **F32), x.new_empty(B, T, 2 * H, **F32), x.new_empty(B, T, 2, 4 * H, **F32),
            cs)


@_op("birnn_layer_bwd")
def birnn_layer_bwd(dout: Tensor, x: Tensor, w_ih: Tensor, w_hh: Tensor, hprev: Tensor, act: Tensor, cs: Tensor,
                    cell: str, H: int, precision: str, need_dx: bool) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    dx, dw_ih, db_ih, dw_hh, db_hh = ag.birnn_bwd_impl(dout, x, w_ih, w_hh, hprev, act,
                                                       cs if cell == "lstm" else None, cell, H, precision, need_dx)
    return (dx if dx is not None else x.new_empty(0)), dw_ih, db_ih, dw_hh, db_hh


@birnn_layer_bwd.register_fake
def _(dout, x, w_ih, w_hh, hprev, act, cs, cell, H, precision, need_dx):
    ng = 2 * (4 if cell == "lstm" else 3) * H
    return (torch.empty_like(x, **F32) if need_dx else x.new_empty(0, **F32), torch.empty_like(w_ih, **F32),
            x.new_empty(ng, **F32), torch.empty_like(w_hh, **F32), x.new_empty(ng, **F32))


def _birnn_setup(ctx, inputs, output):
    x, w_ih, b_ih, w_hh, b_hh, cell, H, precision = inputs
    _, hprev, act, cs = output
    # saved state for the backward, not values a loss may depend on (their gradients would be dropped)
    ctx.mark_non_differentiable(hprev, act, cs)
    ctx.save_for_backward(x, w_ih, w_hh, hprev, act, cs)
    ctx.meta = (cell, H, precision)


def _birnn_backward(ctx, dout, _dhprev, _dact, _dcs):
    x, w_ih, w_hh, hprev, act, cs = ctx.saved_tensors
    cell, H, precision = ctx.meta
    dx, dw_ih, db_ih, dw_hh, db_hh = birnn_layer_bwd(dout.contiguous(), x, w_ih, w_hh, hprev, act, cs, cell, H,
                                                     precision, bool(ctx.needs_input_grad[0]))
    return (dx if ctx.needs_input_grad[0] else None), dw_ih, db_ih, dw_hh, db_hh, None, None, None


birnn_layer.register_autograd(_birnn_backward, setup_context=_birnn_setup)


def birnn(x, w_ih, b_ih, w_hh, b_hh, cell="lstm", H=300, precision="fp32"):
    """One bidirectional layer through ``dl4ss::birnn_layer``: out (B, T, 2H) only."""
    return torch.ops.dl4ss.birnn_layer(x, w_ih, b_ih, w_hh, b_hh, cell, H, precision)[0]


# --------------------------------------------------------------------------- Linear + tanh head
@_op("linear_tanh")
def linear_tanh(x2d: Tensor, w: Tensor, b: Tensor, precision: str) -> Tensor:
    return ops.gemm(ag._c(x2d), ag._c(w), transB=True, bias=ag._c(b), epilogue=ops.EPI_TANH, precision=precision)


@linear_tanh.register_fake
def _(x2d, w, b, precision):
    return x2d.new_empty(x2d.shape[0], w.shape[0], **F32)


@_op("linear_tanh_bwd")
def linear_tanh_bwd(dv: Tensor, x2d: Tensor, w: Tensor, v: Tensor, precision: str,
                    need_dx: bool) -> Tuple[Tensor, Tensor, Tensor]:
    dx, dw, db = ag.linear_tanh_bwd_impl(dv, x2d, w, v, precision, need_dx)
    return (dx if dx is not None else x2d.new_empty(0)), dw, db


@linear_tanh_bwd.register_fake
def _(dv, x2d, w, v, precision, need_dx):
    return ((torch.empty_like(x2d, **F32) if need_dx else x2d.new_empty(0, **F32)), torch.empty_like(w, **F32),
            w.new_empty(w.shape[0], **F32))


def _lt_setup(ctx, inputs, output):
    x2d, w, b, precision = inputs
    ctx.save_for_backward(x2d, w, output)
    ctx.precision = precision


def _lt_backward(ctx, dv):
    x2d, w, v = ctx.saved_tensors
    dx, dw, db = linear_tanh_bwd(dv.contiguous(), x2d, w, v, ctx.precision, bool(ctx.needs_input_grad[0]))
    return (dx if ctx.needs_input_grad[0] else None), dw, db, None


linear_tanh.register_autograd(_lt_backward, setup_context=_lt_setup)


# --------------------------------------------------------------------------- ATTENTION 'dot'
@_op("attention_dot")
def attention_dot(V: Tensor, q: Tensor, crm: bool) -> Tensor:
    return ag.attention_dot_fwd_impl(V, q, crm)


@attention_dot.register_fake
def _(V, q, crm):
    Bq, R, _ = V.shape
    return V.new_empty(Bq, R, 2, **F32) if crm else V.new_empty(Bq, R, **F32)


@_op("attention_dot_bwd")
def attention_dot_bwd(dmask: Tensor, V: Tensor, q: Tensor, mask: Tensor, crm: bool,
                      need_dV: bool) -> Tuple[Tensor, Tensor]:
    masks = [mask[..., h].contiguous() for h in range(2)] if crm else [mask]
    dV, dq = ag.attention_dot_bwd_impl(dmask, V, q, masks, crm, need_dV)
    return (dV if dV is not None else V.new_empty(0)), dq


@attention_dot_bwd.register_fake
def _(dmask, V, q, mask, crm, need_dV):
    return (torch.empty_like(V, **F32) if need_dV else V.new_empty(0, **F32)), torch.empty_like(q, **F32)


def _att_setup(ctx, inputs, output):
    V, q, crm = inputs
    ctx.save_for_backward(V, q, output)
    ctx.crm = crm


def _att_backward(ctx, dmask):
    V, q, mask = ctx.saved_tensors
    dV, dq = attention_dot_bwd(dmask.contiguous(), V, q, mask, ctx.crm, bool(ctx.needs_input_grad[0]))
    return (dV if ctx.needs_input_grad[0] else None), dq, None


attention_dot.register_autograd(_att_backward, setup_context=_att_setup)


# --------------------------------------------------------------------------- top-k speaker mask
@_op("top_k_mask")
def top_k_mask(prob: Tensor, alpha: float, top_k: int) -> Tuple[Tensor, Tensor, Tensor]:
    mask, idx, cnt = ag.top_k_mask_device(prob, alpha, top_k)
    return mask, idx.contiguous(), cnt


@top_k_mask.register_fake
def _(prob, alpha, top_k):
    B, N = prob.shape
    return (prob.new_empty(B, N), prob.new_empty(B, top_k, dtype=torch.int32),
            prob.new_empty(B, dtype=torch.int32))


OPS = ("stft_mag", "stft_complex", "istft", "istft_apply", "mix_sources", "birnn_layer", "birnn_layer_bwd",
       "linear_tanh", "linear_tanh_bwd", "attention_dot", "attention_dot_bwd", "top_k_mask")
