"""torch.autograd.Functions over the HIP kernels, for the reference-API modules
(``dl4ss_amd.compat.myNet``): a driver that composes MIX_SPEECH / ATTENTION /
SPEECH_EMBEDDING / ADDJUST with torch autograd (as the reference's ``main_run_*``
scripts do) runs the recurrence, the GEMMs, the attention and the query gather
on the gfx950 kernels.  The fused single-call training step is
``dl4ss_amd.engine.SepTrainer``; these Functions are the modular path.

Every tensor reaching a kernel must be a contiguous fp32 CUDA tensor (``_lib.ptr``
enforces it); there is no CPU fallback.
"""
import ctypes

import torch

from . import _lib, ops

CELLS = {"lstm": 0, "gru": 1}


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def _check_status(status, what):
    s = int(status.item())
    if s != 0:
        raise RuntimeError(f"{what}: BiRNN hand-off timed out (status {s})")


def birnn_fwd_impl(x, w_ih, b_ih, w_hh, b_hh, cell, H, precision):
    """One bidirectional layer's forward: (out (B,T,2H), hprev, act, cs or None).  Shared by
    BiRNNLayerFn and the dl4ss::birnn_layer custom op (dl4ss_amd.library)."""
    x = _c(x)
    B, T, D = x.shape
    cid = CELLS[cell]
    dev = x.device
    G = ops.gemm(x.view(B * T, D), _c(w_ih), transB=True, bias=_c(b_ih), precision=precision)
    out = torch.empty(B, T, 2 * H, device=dev)
    hprev = torch.empty_like(out)
    act = torch.empty(B, T, 2, 4 * H, device=dev)
    cs = torch.empty(B, T, 2, H, device=dev) if cell == "lstm" else None
    wsn = _birnn_ws_bytes(cid, B, H)
    ws = torch.empty((wsn + 7) // 8, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.call("dl4ss_birnn_fwd", cid, ops.PREC[precision], B, T, H, _lib.ptr(G), _lib.ptr(_c(w_hh)),
              _lib.ptr(_c(b_hh)), _lib.ptr(out), _lib.ptr(hprev), _lib.ptr(act),
              _lib.ptr(cs) if cs is not None else None, _lib.ptr(ws), wsn, _lib.ptr(status), _lib.stream_ptr())
    _check_status(status, "dl4ss_birnn_fwd")
    return out, hprev, act, cs


def _birnn_ws_bytes(cid, B, H):
    wsn = _lib.query("dl4ss_birnn_workspace_bytes", cid, B, H)
    if wsn < 0:
        raise RuntimeError(f"BiRNN shape unsupported (B={B}, H={H})")
    return wsn


def birnn_bwd_impl(dout, x, w_ih, w_hh, hprev, act, cs, cell, H, precision, need_dx=True):
    """BPTT + the layer's weight / bias / input gradients: (dx or None, dw_ih, db_ih, dw_hh, db_hh)."""
    B, T, D = x.shape
    dev = x.device
    NGH = (4 if cell == "lstm" else 3) * H
    wsn = _birnn_ws_bytes(CELLS[cell], B, H)
    dout = _c(dout.float())
    dG = torch.empty(B * T, 2 * NGH, device=dev)
    dGh = torch.empty_like(dG) if cell == "gru" else None
    ws = torch.empty((wsn + 7) // 8, dtype=torch.int64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.call("dl4ss_birnn_bwd", CELLS[cell], ops.PREC[precision], B, T, H, _lib.ptr(dout), None,
              _lib.ptr(_c(w_hh)), _lib.ptr(act), _lib.ptr(cs) if cell == "lstm" else None, _lib.ptr(hprev),
              _lib.ptr(dG), _lib.ptr(dGh) if dGh is not None else None, _lib.ptr(ws), wsn, _lib.ptr(status),
              _lib.stream_ptr())
    _check_status(status, "dl4ss_birnn_bwd")
    dGh = dG if dGh is None else dGh
    w_ih = _c(w_ih)
    x2 = _c(x).view(B * T, D)
    dx = ops.gemm(dG, w_ih, precision=precision).view(B, T, D) if need_dx else None
    dw_ih = torch.zeros_like(w_ih)
    ops.gemm(dG, x2, transA=True, out=dw_ih, beta=1.0, splitk="auto", precision=precision)
    db_ih = torch.zeros(2 * NGH, device=dev)
    ops.colsum(dG, db_ih)
    dw_hh = torch.zeros_like(w_hh)
    hp = hprev.view(B * T, 2 * H)
    for d in range(2):
        ops.gemm(dGh[:, d * NGH:(d + 1) * NGH], hp[:, d * H:(d + 1) * H], transA=True,
                 out=dw_hh[d * NGH:(d + 1) * NGH], beta=1.0, splitk="auto", precision=precision)
    db_hh = torch.zeros(2 * NGH, device=dev)
    ops.colsum(dGh, db_hh)
    return dx, dw_ih, db_ih, dw_hh, db_hh


class BiRNNLayerFn(torch.autograd.Function):
    """One bidirectional LSTM/GRU layer (torch gate order / two-bias semantics).

    x (B,T,D); w_ih (2*G*H, D), b_ih (2*G*H), w_hh (2*G*H, H), b_hh (2*G*H) with the
    forward direction's rows first (G = 4 LSTM / 3 GRU)  ->  out (B,T,2H) = [fwd | rev].
    Replaces one layer of nn.LSTM / nn.GRU(batch_first, bidirectional)
    (TDAA_beta/main_run_sstune_EvalVer.py:282-293, Torch_multi/main_run.py:263-273).
    """

    @staticmethod
    def forward(ctx, x, w_ih, b_ih, w_hh, b_hh, cell, H, precision):
        out, hprev, act, cs = birnn_fwd_impl(x, w_ih, b_ih, w_hh, b_hh, cell, H, precision)
        ctx.save_for_backward(_c(x), _c(w_ih), _c(w_hh), hprev, act, cs if cs is not None else act)
        ctx.meta = (cell, H, precision)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, w_ih, w_hh, hprev, act, cs = ctx.saved_tensors
        cell, H, precision = ctx.meta
        dx, dw_ih, db_ih, dw_hh, db_hh = birnn_bwd_impl(dout, x, w_ih, w_hh, hprev, act,
                                                        cs if cell == "lstm" else None, cell, H, precision,
                                                        bool(ctx.needs_input_grad[0]))
        return dx, dw_ih, db_ih, dw_hh, db_hh, None, None, None


def linear_tanh_bwd_impl(dv, x2d, w, v, precision, need_dx=True):
    """(dx or None, dW, db) of V = tanh(x W^T + b), from the saved V."""
    dv = _c(dv.float())
    dpre = torch.empty_like(v)
    _lib.call("dl4ss_tanh_bwd", _lib.ptr(v), _lib.ptr(dv), _lib.ptr(dpre), v.numel(), _lib.stream_ptr())
    dw = torch.zeros_like(w)
    ops.gemm(dpre, x2d, transA=True, out=dw, beta=1.0, splitk="auto", precision=precision)
    db = torch.zeros(w.shape[0], device=w.device)
    ops.colsum(dpre, db)
    dx = ops.gemm(dpre, w, precision=precision) if need_dx else None
    return dx, dw, db


class LinearTanhFn(torch.autograd.Function):
    """V = tanh(x W^T + b), the MIX_SPEECH output head (EvalVer.py:290,298-299)."""

    @staticmethod
    def forward(ctx, x2d, w, b, precision):
        x2d, w = _c(x2d), _c(w)
        v = ops.gemm(x2d, w, transB=True, bias=_c(b), epilogue=ops.EPI_TANH, precision=precision)
        ctx.save_for_backward(x2d, w, v)
        ctx.precision = precision
        return v

    @staticmethod
    def backward(ctx, dv):
        x2d, w, v = ctx.saved_tensors
        dx, dw, db = linear_tanh_bwd_impl(dv, x2d, w, v, ctx.precision, bool(ctx.needs_input_grad[0]))
        return dx, dw, db, None


class LinearFn(torch.autograd.Function):
    """y = x W^T (+ b) on the GEMM kernel (ADDJUST's bias-free Linear, EvalVer.py:366;
    the classifier head)."""

    @staticmethod
    def forward(ctx, x2d, w, b, precision):
        x2d, w = _c(x2d.float()), _c(w)
        y = ops.gemm(x2d, w, transB=True, bias=_c(b) if b is not None else None, precision=precision)
        ctx.save_for_backward(x2d, w)
        ctx.precision, ctx.has_b = precision, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x2d, w = ctx.saved_tensors
        dy = _c(dy.float())
        dw = ops.gemm(dy, x2d, transA=True, precision=ctx.precision)
        db = None
        if ctx.has_b:
            db = torch.zeros(w.shape[0], device=w.device)
            ops.colsum(dy, db)
        dx = ops.gemm(dy, w, precision=ctx.precision) if ctx.needs_input_grad[0] else None
        return dx, dw, db, None


def attention_dot_fwd_impl(V, q, crm):
    """mask (Bq,R) = sigmoid(V . q), or (Bq,R,2) = 10 tanh(V . q_half) for the cRM branch."""
    return torch.stack(_attention_dot_masks(V, q, crm), dim=-1) if crm else _attention_dot_masks(V, q, crm)[0]


def _attention_dot_masks(V, q, crm):
    V, q = _c(V.float()), _c(q.float())
    Bq, R, E = V.shape
    st = _lib.stream_ptr()
    masks = []
    for h in range(2 if crm else 1):
        m = torch.empty(Bq, R, device=V.device)
        _lib.call("dl4ss_attn_dot_fwd", _lib.ptr(V), ctypes.c_void_p(q.data_ptr() + 4 * h * E), q.shape[1], Bq, R,
                  E, int(crm), _lib.ptr(m), st)
        masks.append(m)
    return masks


def attention_dot_bwd_impl(dmask, V, q, masks, crm, need_dV=True):
    """(dV or None, dq) from the per-half masks of the forward."""
    V, q = _c(V.float()), _c(q.float())
    Bq, R, E = V.shape
    st = _lib.stream_ptr()
    dV = torch.zeros_like(V) if need_dV else None
    nblk = _lib.query("dl4ss_attn_dot_nblk", R)
    part = torch.empty(Bq * nblk * E, device=V.device)
    dq = torch.zeros_like(q)
    dqh = torch.empty(Bq, E, device=V.device)
    for h, m in enumerate(masks):
        dm = _c(dmask[..., h].float()) if crm else _c(dmask.float())
        _lib.call("dl4ss_attn_dot_bwd", _lib.ptr(V), ctypes.c_void_p(q.data_ptr() + 4 * h * E), q.shape[1],
                  _lib.ptr(m), _lib.ptr(dm), Bq, R, E, int(crm), _lib.ptr(dV) if dV is not None else None,
                  _lib.ptr(part), _lib.ptr(dqh), st)
        dq[:, h * E:(h + 1) * E] = dqh
    return dV, dq


class AttentionDotFn(torch.autograd.Function):
    """ATTENTION 'dot' (EvalVer.py:216-226): mask (Bq,R) = sigmoid(V (Bq,R,E) . q (Bq,E));
    crm=True: the cRM branch (cRM_EvalVer.py:259-271), q (Bq,2E) split in halves,
    mask (Bq,R,2) = 10 tanh(V . q_half)."""

    @staticmethod
    def forward(ctx, V, q, crm):
        V, q = _c(V.float()), _c(q.float())
        masks = _attention_dot_masks(V, q, crm)
        ctx.save_for_backward(V, q, *masks)
        ctx.crm = crm
        return torch.stack(masks, dim=-1) if crm else masks[0]

    @staticmethod
    def backward(ctx, dmask):
        V, q, *masks = ctx.saved_tensors
        dV, dq = attention_dot_bwd_impl(dmask, V, q, masks, ctx.crm, bool(ctx.needs_input_grad[0]))
        return dV, dq, None


class EmbeddingGatherFn(torch.autograd.Function):
    """q (B,K,W) = Emb[idx]: SPEECH_EMBEDDING gather (EvalVer.py:355-360)."""

    @staticmethod
    def forward(ctx, emb, idx):
        emb = _c(emb)
        idx = _c(idx.to(torch.int32))
        B, K = idx.shape
        W = emb.shape[1]
        q = torch.empty(B, K, W, device=emb.device)
        # query kernel without ADJUST: a pure gather (h / mean unused)
        _lib.call("dl4ss_query_fwd", _lib.ptr(emb), B, 1, 1, _lib.ptr(idx), _lib.ptr(emb), None, K, W, _lib.ptr(q),
                  None, _lib.stream_ptr())
        ctx.save_for_backward(idx)
        ctx.shape = emb.shape
        return q

    @staticmethod
    def backward(ctx, dq):
        (idx,) = ctx.saved_tensors
        B, K = idx.shape
        n, W = ctx.shape
        demb = torch.zeros(n, W, device=dq.device)
        dq = _c(dq.float())
        _lib.call("dl4ss_query_bwd", _lib.ptr(dq), B, 1, 1, _lib.ptr(idx), None, None, None, K, W, _lib.ptr(demb),
                  None, None, _lib.stream_ptr())
        return demb, None


def top_k_mask_device(prob, alpha, top_k):
    """(mask (B,N) float, idx (B,top_k) int32 ascending, -1 padded, count (B,) int32) on device."""
    prob = _c(prob.float())
    B, N = prob.shape
    mask = torch.empty(B, N, device=prob.device)
    idx = torch.empty(B, max(top_k, 1), dtype=torch.int32, device=prob.device)
    cnt = torch.empty(B, dtype=torch.int32, device=prob.device)
    _lib.call("dl4ss_top_k_mask", _lib.ptr(prob), B, N, float(alpha), int(top_k), _lib.ptr(mask), _lib.ptr(idx),
              _lib.ptr(cnt), _lib.stream_ptr())
    return mask, idx[:, :top_k], cnt
