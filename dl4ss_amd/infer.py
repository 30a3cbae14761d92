"""Inference paths on the HIP kernels: the speaker classifier, the mask net forward, the
test-mode speaker selection and the recursive extraction loop (SURVEY R9 classifier, R17,
section 8f f1).

* ``ClassifierNet`` -- ``MIX_SPEECH_classifier`` (``Torch_multi/main_run_multi_selfSS_recuReal_GRID.py:178-199``,
  ``TDAA_beta/main_run_sstune_EvalVer.py:305-326``): BiLSTM(129, 600, 3 layers) -> mean over t ->
  Linear(1200, N_lab) -> sigmoid.  Flat fp32 parameters under the reference ``state_dict``
  names (``layer.weight_ih_l0``, ..., ``Linear.weight``), so a reference checkpoint loads
  directly.  Its H = 600 recurrence runs the forward-only large-H plan of ``birnn.hip``.
* ``MaskNetForward`` -- ``MIX_SPEECH`` forward only (V = tanh(Linear(BiRNN(X)))) on a ``SepNet``.
* ``RecursiveExtractor`` -- the recursive extraction loop of ``GRID.py:383-475`` (SURVEY section
  3 (E)): classifier -> on-device choice of the first not-yet-extracted speaker among the
  top 3 (``dl4ss_classifier_select``) -> attention mask -> residual (1 - M) X -> again; then
  the masks of every extracted speaker on the original mixture.  The reference round-trips
  the residual through the host and syncs on every speaker choice (``GRID.py:391-444``);
  here every step stays on the device and the host reads the result once.
* ``select_speakers`` -- the test-mode selection of ``EvalVer.py:436-442``:
  ``top_k_mask(classifier(X), alpha=-0.5, top_k=2)`` in label order.

Everything arithmetic is a C-ABI call into ``libdl4ss_hip.so``; torch owns the buffers.
"""
import ctypes
import math

import torch

from . import _lib, ops
from .engine import CELLS, _ngate


# split-precision operand images (dl4ss_f32_to_bf16_hilo): [x_hi | x_lo | x_hi] . [w_hi | w_hi | w_lo]
A_SPLIT, W_SPLIT = 0b010, 0b100


def _p8(n):
    return (n + 7) // 8 * 8


def _hilo(x, y, segw, pattern):
    """y = the three-segment split image of the fp32 rows x (segments of segw, hi / lo by pattern)."""
    _lib.call("dl4ss_f32_to_bf16_hilo", _lib.ptr(x, True), x.stride(0), x.shape[0], x.shape[1], _lib.ptr(y),
              y.stride(0), segw, 3, pattern, _lib.stream_ptr())


class _SplitWeights:
    """The [w_hi | w_hi | w_lo] images of a net's weights for the "bf16s" GEMMs, converted once per
    parameter generation: reused while (net.generation, net.flat._version) is what it was when they
    were made (engine.SepNet's contract for writes that bypass torch's version counter)."""

    def __init__(self, net):
        self.net, self.key, self.img = net, None, {}

    def get(self, name, w):
        key = (getattr(self.net, "generation", 0), self.net.flat._version)
        if key != self.key:
            self.img, self.key = {}, key
        if name not in self.img:
            seg = _p8(w.shape[1])
            y = torch.empty(w.shape[0], 3 * seg, device=w.device, dtype=torch.bfloat16)
            _hilo(w, y, seg, W_SPLIT)
            self.img[name] = y
        return self.img[name]


class _BiRNNStack:
    """Forward-only stacked bidirectional LSTM / GRU (input GEMM + persistent recurrence per
    layer) with its buffers for one (B, T)."""

    def __init__(self, cell, hidden, num_layers, B, T, device):
        self.cell, self.H, self.L, self.B, self.T = cell, hidden, num_layers, B, T
        H = hidden
        f32 = dict(device=device, dtype=torch.float32)
        NGH = _ngate(cell) * H
        self.G = torch.empty(B * T, 2 * NGH, **f32)
        self.out = [torch.empty(B, T, 2 * H, **f32) for _ in range(min(2, num_layers))]
        self.hprev = torch.empty(B, T, 2 * H, **f32)
        self.act = torch.empty(B, T, 2, 4 * H, **f32)
        self.cs = torch.empty(B, T, 2, H, **f32) if cell == "lstm" else None
        wsn = _lib.query("dl4ss_birnn_workspace_bytes", CELLS[cell], B, H)
        if wsn < 0:
            raise RuntimeError(f"BiRNN shape unsupported (cell={cell}, B={B}, H={H})")
        self.wsn = wsn
        self.ws = torch.empty((wsn + 7) // 8, dtype=torch.int64, device=device)
        self.status = torch.zeros(1, dtype=torch.int32, device=device)

    def run(self, x2d, cat_view, precision, rnn_precision=None, split_w=None):
        """x2d (B*T, D0) fp32 -> (B, T, 2H); cat_view(kind, l) gives the [fwd; reverse]
        parameter of layer l (``weight_ih`` / ``weight_hh`` / ``bias_ih`` / ``bias_hh``).
        ``precision``: the input-projection GEMMs -- "fp32", "bf16", or "bf16s": one bf16 LDS-DMA
        GEMM over split operands (K' = 3 K, fp32-accurate to ~2^-16; the training step's bf16s
        forward GEMMs), with ``split_w`` (a _SplitWeights) holding the weight images;
        ``rnn_precision`` (default: the same; "bf16" for bf16s) the recurrent matvec."""
        B, T, H = self.B, self.T, self.H
        rnn_precision = rnn_precision or ("bf16" if precision == "bf16s" else precision)
        st = _lib.stream_ptr()
        x = x2d
        out = None
        for l in range(self.L):
            if precision == "bf16s":
                seg = _p8(x.shape[1])
                xs = self._xs(B * T, 3 * seg, x.device)
                _hilo(x, xs, seg, A_SPLIT)
                ops.gemm_bf16_gl(xs, split_w.get(f"weight_ih_l{l}", cat_view("weight_ih", l)), transB=True,
                                 bias=cat_view("bias_ih", l), out=self.G)
            else:
                ops.gemm(x, cat_view("weight_ih", l), transB=True, bias=cat_view("bias_ih", l), out=self.G,
                         precision=precision)
            out = self.out[l % 2]
            _lib.call("dl4ss_birnn_fwd", CELLS[self.cell], ops.PREC[rnn_precision], B, T, H, _lib.ptr(self.G),
                      _lib.ptr(cat_view("weight_hh", l)), _lib.ptr(cat_view("bias_hh", l)), _lib.ptr(out),
                      _lib.ptr(self.hprev), _lib.ptr(self.act), _lib.ptr(self.cs) if self.cs is not None else None,
                      _lib.ptr(self.ws), self.wsn, _lib.ptr(self.status), st)
            x = out.view(B * T, 2 * H)
        return out

    def _xs(self, rows, cols, device):
        """the split image of a layer input, (rows, cols) bf16 (one buffer, grown to the widest layer)"""
        buf = getattr(self, "_xs_buf", None)
        if buf is None or buf.numel() < rows * cols:
            buf = self._xs_buf = torch.empty(rows * cols, device=device, dtype=torch.bfloat16)
        return buf[:rows * cols].view(rows, cols)

    def check(self):
        s = int(self.status.item())
        if s != 0:
            raise RuntimeError(f"BiRNN hand-off timed out (status {s})")


class ClassifierNet:
    """Parameters of MIX_SPEECH_classifier, flat fp32 with the reference names."""

    def __init__(self, input_fre=129, hidden=600, num_layers=3, num_labels=101, device="cuda", seed=1):
        self.F, self.H, self.L, self.num_labels = input_fre, hidden, num_layers, num_labels
        NGH = 4 * hidden
        specs = []
        for l in range(num_layers):
            D = input_fre if l == 0 else 2 * hidden
            for kind, shape in (("weight_ih", (NGH, D)), ("weight_hh", (NGH, hidden)), ("bias_ih", (NGH,)),
                                ("bias_hh", (NGH,))):
                specs.append((f"layer.{kind}_l{l}", shape))
                specs.append((f"layer.{kind}_l{l}_reverse", shape))
        specs += [("Linear.weight", (num_labels, 2 * hidden)), ("Linear.bias", (num_labels,))]
        self.specs = specs
        self.offsets = {}
        off = 0
        for name, shape in specs:
            self.offsets[name] = (off, shape)
            off += (math.prod(shape) + 3) // 4 * 4  # 16-B aligned views
        self.device = torch.device(device)
        self.flat = torch.zeros(off, device=self.device, dtype=torch.float32)
        self.reset_parameters(seed)

    def view(self, name):
        off, shape = self.offsets[name]
        return self.flat[off:off + math.prod(shape)].view(shape)

    def cat_view(self, kind, l):
        """[fwd; reverse] of layer l (adjacent in the flat buffer by construction)."""
        a = self.view(f"layer.{kind}_l{l}")
        off = self.offsets[f"layer.{kind}_l{l}"][0]
        n = a.numel()
        v = self.flat[off:off + 2 * n]
        return v.view(2 * a.shape[0], *a.shape[1:]) if a.dim() == 2 else v

    def reset_parameters(self, seed=1):
        """torch defaults: nn.LSTM U(+-1/sqrt(H)), nn.Linear U(+-1/sqrt(fan_in))."""
        g = torch.Generator().manual_seed(seed)
        for name, shape in self.specs:
            k = 1.0 / math.sqrt(self.H if name.startswith("layer.") else 2 * self.H)
            self.view(name).copy_(torch.empty(shape).uniform_(-k, k, generator=g))

    def load_state_dict(self, sd):
        for name, _ in self.specs:
            self.view(name).copy_(sd[name].to(torch.float32))

    def state_dict(self):
        return {name: self.view(name).detach().clone() for name, _ in self.specs}


class ClassifierForward:
    """classifier(X) on the HIP path for one (B, T): logits / probabilities (B, N_lab)."""

    def __init__(self, cnet, B, T, precision="fp32"):
        self.net, self.B, self.T, self.precision = cnet, B, T, precision
        dev = cnet.device
        self.stack = _BiRNNStack("lstm", cnet.H, cnet.L, B, T, dev)
        self.mean = torch.empty(B, 2 * cnet.H, device=dev)
        self.logits = torch.empty(B, cnet.num_labels, device=dev)
        self.prob = torch.empty(B, cnet.num_labels, device=dev)

    def logits_of(self, feats):
        """feats (B, T, F) fp32 -> logits (B, N_lab) (buffer reused by the next call)."""
        B, T = self.B, self.T
        h = self.stack.run(feats.reshape(B * T, -1), self.net.cat_view, self.precision)
        _lib.call("dl4ss_time_mean", _lib.ptr(h), B, T, 2 * self.net.H, _lib.ptr(self.mean), _lib.stream_ptr())
        ops.gemm(self.mean, self.net.view("Linear.weight"), transB=True, bias=self.net.view("Linear.bias"),
                 out=self.logits, precision=self.precision)
        return self.logits

    def select(self, feats, alpha, top_k, prev=None, chosen=None, sort_index=None):
        """Probabilities (into self.prob) and the speaker choice of one recursion step."""
        logits = self.logits_of(feats)
        n_prev = 0 if prev is None else prev.shape[0]
        _lib.call("dl4ss_classifier_select", _lib.ptr(logits), self.B, self.net.num_labels, float(alpha), int(top_k),
                  _lib.ptr(prev), n_prev, _lib.ptr(self.prob), _lib.ptr(sort_index), _lib.ptr(chosen),
                  _lib.stream_ptr())
        return self.prob

    def __call__(self, feats):
        return self.select(feats, 0.0, 1)


class MaskNetForward:
    """MIX_SPEECH forward on a SepNet: V (B*T, F*E) = tanh(Linear(BiRNN(X))).  ``precision``: the
    GEMMs (input projections, Linear; "fp32", "bf16" or the split-operand "bf16s");
    ``rnn_precision`` (default: the same, "bf16" for bf16s): the recurrence."""

    def __init__(self, net, B, T, precision="fp32", rnn_precision=None):
        self.net, self.B, self.T, self.precision = net, B, T, precision
        self.rnn_precision = rnn_precision or ("bf16" if precision == "bf16s" else precision)
        self.stack = _BiRNNStack(net.cell, net.H, net.L, B, T, net.device)
        self.split_w = _SplitWeights(net) if precision == "bf16s" else None
        self.h = None

    def __call__(self, feats, out):
        B, T, net = self.B, self.T, self.net
        self.h = self.stack.run(feats.reshape(B * T, -1), net.cat_view, self.precision, self.rnn_precision,
                                split_w=self.split_w)
        h2 = self.h.view(B * T, 2 * net.H)
        if self.precision == "bf16s":
            seg = _p8(2 * net.H)
            hs = self.stack._xs(B * T, 3 * seg, h2.device)
            _hilo(h2, hs, seg, A_SPLIT)
            ops.gemm_bf16_gl(hs, self.split_w.get("mix.Linear.weight", net.view("mix.Linear.weight")), transB=True,
                             bias=net.view("mix.Linear.bias"), epilogue=ops.EPI_TANH, out=out)
            return out
        ops.gemm(h2, net.view("mix.Linear.weight"), transB=True,
                 bias=net.view("mix.Linear.bias"), epilogue=ops.EPI_TANH, out=out, precision=self.precision)
        return out


def select_speakers(classifier, feats, alpha=-0.5, top_k=2):
    """Test-mode speaker selection (EvalVer.py:436-442): top_k_mask(classifier(X), alpha, top_k)
    -> (multi-hot mask (B, N_lab), ids (B, top_k) ascending / -1 padded, count (B,)), on device."""
    prob = classifier(feats)
    B, N = prob.shape
    mask = torch.empty(B, N, device=prob.device)
    idx = torch.empty(B, top_k, dtype=torch.int32, device=prob.device)
    cnt = torch.empty(B, dtype=torch.int32, device=prob.device)
    _lib.call("dl4ss_top_k_mask", _lib.ptr(prob), B, N, float(alpha), int(top_k), _lib.ptr(mask), _lib.ptr(idx),
              _lib.ptr(cnt), _lib.stream_ptr())
    return mask, idx, cnt


class RecursiveExtractor:
    """The recursive extraction loop of GRID.py:383-475 for a batch of B independent rows
    (the reference runs B = 1).  ``net``: the GRID mask net (SepNet, BiGRU-2L,
    no ADJUST; its ``emb.layer.weight`` is the speaker embedding); ``cnet``: ClassifierNet.

    ``precision``: "fp32" (exact GEMMs and recurrences), "bf16" (bf16 operands everywhere, fp32
    accumulate and state), "bf16s" -- the mask net's GEMMs (input projections, Linear -> V) as ONE
    bf16 GEMM each over split operands (hi + lo bf16, K' = 3 K: fp32-accurate to ~2^-16, at bf16
    MFMA speed) with its recurrence on bf16 operands, the classifier in bf16 -- or "mixed", the same
    with the mask net's GEMMs on the exact fp32 MFMA (half the speed of bf16s, round 5).  The masks are
    sigmoids of V . emb with N(0,1) speaker embeddings and no ADDJUST: every bf16-rounded GEMM operand
    of the mask net costs ~1e-3 of masked-magnitude error (tools/bf16_budget.py on the same BiGRU-2L
    net), the recurrence ~0.3e-3, so "bf16s" (and "mixed") are the modes within the north-star 1e-3
    (C5 in DESIGN.md section 6; quoted in bf16s from round 6).  The classifier only decides the speaker
    ids (its bf16 probabilities are within ~1e-4 of fp32)."""

    MODES = {"fp32": ("fp32", "fp32", "fp32"), "bf16": ("bf16", "bf16", "bf16"), "mixed": ("fp32", "bf16", "bf16"),
             "bf16s": ("bf16s", "bf16", "bf16")}

    def __init__(self, net, cnet, B, T, precision="fp32", alpha=-0.3, top_k=3, max_steps=2):
        if net.E != 50 or net.crm:
            raise ValueError("the recursive path is the magnitude-mask 'dot' attention with E = 50")
        if precision not in self.MODES:
            raise ValueError(f"precision {precision!r}: expected one of {sorted(self.MODES)}")
        mask_gemm, mask_rnn, cls_prec = self.MODES[precision]
        self.precision = precision
        self.net, self.cnet, self.B, self.T = net, cnet, B, T
        self.alpha, self.top_k, self.S = alpha, top_k, max_steps
        dev = net.device
        F, E = net.F, net.E
        f32 = dict(device=dev, dtype=torch.float32)
        self.mask_net = MaskNetForward(net, B, T, mask_gemm, mask_rnn)
        self.classifier = ClassifierForward(cnet, B, T, cls_prec)
        self.V0 = torch.empty(B * T, F * E, **f32)
        self.V = torch.empty(B * T, F * E, **f32)
        self.feats = [torch.empty(B, T, F, **f32) for _ in range(2)]
        self.chosen = torch.full((max_steps, B), -1, dtype=torch.int32, device=dev)
        self.sort_index = torch.empty(max_steps, B, top_k, dtype=torch.int32, device=dev)
        self.q = torch.empty(B, 1, E, **f32)
        self.qf = torch.empty(B, max_steps, E, **f32)
        self.step_mask = torch.empty(B, T, F, **f32)
        self.step_pred = torch.empty(max_steps, B, T, F, **f32)
        self.masks = torch.empty(B, max_steps, T, F, **f32)
        self.probs = torch.empty(max_steps, B, cnet.num_labels, **f32)

    def _gather(self, idx, K, out):
        """out (B, K, E) = emb[idx (B, K)] (zero rows for idx -1): SPEECH_EMBEDDING, GRID.py:208-213."""
        emb = _lib.ptr(self.net.view("emb.layer.weight"))
        _lib.call("dl4ss_query_fwd", emb, self.B, 1, 1, _lib.ptr(idx), emb, None, K, self.net.E, _lib.ptr(out), None,
                  _lib.stream_ptr())

    def _attend(self, V, q, out):
        """out[b, k] = sigmoid(V[b] . q[b, k]) for q (B, K, E), out (B, K, T, F) contiguous: K launches
        over the same V (no expanded copy), row stride K*T*F."""
        R, E = self.T * self.net.F, self.net.E
        K = q.shape[1]
        assert q.is_contiguous() and out.is_contiguous() and out.numel() == self.B * K * R
        for k in range(K):
            _lib.call("dl4ss_attn_dot_fwd_ex", _lib.ptr(V), ctypes.c_void_p(q.data_ptr() + 4 * k * E), K * E, self.B,
                      R, E, 0, ctypes.c_void_p(out.data_ptr() + 4 * k * R), K * R, _lib.stream_ptr())

    def run(self, feats):
        """feats (B, T, F) fp32 on the device (magnitude spectrogram of the mixtures).
        Returns a dict of device tensors: spk (B, S) int32 (-1 = none), masks (B, S, T, F) on
        the original mixture, step_pred (S, B, T, F) (each step's predict_multi_map),
        probs (S, B, N_lab)."""
        B, T, F, S = self.B, self.T, self.net.F, self.S
        R = T * F
        X = feats.contiguous()
        self.mask_net(X, self.V0)
        self.chosen.fill_(-1)
        now, V = X, self.V0
        for s in range(S):
            self.classifier.select(now, self.alpha, self.top_k, prev=self.chosen[:s] if s else None,
                                   chosen=self.chosen[s], sort_index=self.sort_index[s])
            self.probs[s].copy_(self.classifier.prob)
            self._gather(self.chosen[s], 1, self.q)
            self._attend(V, self.q, self.step_mask)
            nxt = self.feats[s % 2]
            _lib.call("dl4ss_mask_split", _lib.ptr(self.step_mask), _lib.ptr(now), B * R, _lib.ptr(self.step_pred[s]),
                      _lib.ptr(nxt) if s + 1 < S else None, _lib.stream_ptr())
            if s + 1 < S:
                now = nxt
                V = self.mask_net(now, self.V)
        # masks of every extracted speaker on the original mixture (GRID.py:455-475)
        spk = self.chosen.t().contiguous()
        self._gather(spk, S, self.qf)
        self._attend(self.V0, self.qf, self.masks)
        for st in (self.mask_net.stack, self.classifier.stack):
            st.check()
        return dict(spk=spk, masks=self.masks, step_pred=self.step_pred, probs=self.probs,
                    sort_index=self.sort_index)
