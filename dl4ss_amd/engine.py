"""The separation training step on the HIP path (host orchestration).

One step (``TDAA_beta/main_run_sstune_EvalVer.py:586-675``,
``main_run_sstune_cRM_EvalVer.py:639-752``, ``Torch_multi/main_run.py:453-522``):

    raw sources -> normalise/gain/mix (R1) -> STFT of mixture and sources (R2-R4)
    -> stacked BiLSTM/BiGRU (R8/R9) -> Linear + tanh -> V (B,T,F,E)
    -> speaker queries (embedding + ADDJUST, R7/R10)
    -> fused mask attention + label-ordered / PIT / cRM loss + backward (R11-R14)
    -> BPTT, weight gradients -> (optional DP all-reduce) -> Adam (R15)

Every arithmetic step is a C-ABI call into ``libdl4ss_hip.so``; torch only owns
device memory, streams and (for DP) the collective.  All parameters live in one
flat fp32 buffer (views carry the reference ``state_dict`` key names, so a
reference / oracle state dict loads directly) and all gradients in a second
flat buffer: one all-reduce and one Adam launch per step.
"""
import ctypes
import math
import os

import torch

from . import _lib, ops

CELLS = {"lstm": 0, "gru": 1}
WS_ZEROED = 0x100  # DL4SS_RNN_WS_ZEROED (include/dl4ss_hip.h)
DGH_PAD8 = 0x200  # DL4SS_RNN_DGH_PAD8
DEFER_BIAS = 0x400  # DL4SS_RNN_DEFER_BIAS


def DOUT_SLABS(n):  # DL4SS_RNN_DOUT_SLABS(S): the BPTT sums dOut's S split-K slabs itself
    return ((n - 1) & 3) << 12


def _ngate(cell):
    return 4 if cell == "lstm" else 3


class SepNet:
    """Trainable parameters of the mask network, flat fp32 with named views."""

    def __init__(self, cell="lstm", num_layers=4, hidden=300, emb=50, num_labels=101, input_fre=129, crm=False,
                 adjust=True, device="cuda", seed=1):
        self.cell, self.L, self.H, self.E = cell, num_layers, hidden, emb
        self.F, self.num_labels, self.crm, self.adjust = input_fre, num_labels, crm, adjust
        self.W = 2 * emb if crm else emb
        NGH = _ngate(cell) * hidden
        specs = []
        for l in range(num_layers):
            D = input_fre if l == 0 else 2 * hidden
            for kind, shape in (("weight_ih", (NGH, D)), ("weight_hh", (NGH, hidden)), ("bias_ih", (NGH,)),
                                ("bias_hh", (NGH,))):
                specs.append((f"mix.layer.{kind}_l{l}", shape))
                specs.append((f"mix.layer.{kind}_l{l}_reverse", shape))
        specs += [("mix.Linear.weight", (input_fre * emb, 2 * hidden)), ("mix.Linear.bias", (input_fre * emb,)),
                  ("emb.layer.weight", (num_labels, self.W))]
        if adjust:
            specs.append(("adj.layer.weight", (self.W, 2 * hidden + self.W)))
        self.specs = specs
        self.offsets = {}
        off = 0
        for name, shape in specs:
            n = math.prod(shape)
            self.offsets[name] = (off, shape)
            off += (n + 3) // 4 * 4  # 16-B aligned views
        self.numel = off
        self.device = torch.device(device)
        self.flat = torch.zeros(off, device=self.device, dtype=torch.float32)
        # the flat gradient behind one 16-B slot: slot 0 carries each rank's hand-off status flag
        # through the gradient all-reduce (SepTrainer.allreduce), so every rank's guarded Adam
        # refuses the same steps.  Layout [flag | layers | Linear, emb, adj]: the data-parallel
        # step's two buckets are the contiguous ranges in front of and behind the Linear weight
        # (bucket_split)
        self.grad_ext = torch.zeros(off + 4, device=self.device, dtype=torch.float32)
        self.grad = self.grad_ext[4:]
        self.dp_flag = self.grad_ext[0:1]
        # generation of `flat` for writers torch's version counter does not see (the device-side
        # Adam of any trainer on this net, a raw-pointer kernel, a collective): every such write
        # bumps it (params_changed()), and a trainer trusts its bf16 weight copies only while
        # (generation, flat._version) is what it was when the copies were made
        self.generation = 0
        self.reset_parameters(seed)

    def params_changed(self):
        """Declare that `flat` was rewritten by means that may bypass torch's version counter:
        every trainer on this net re-derives its bf16 weight copies on its next step."""
        self.generation += 1

    def view(self, name, buf=None):
        off, shape = self.offsets[name]
        return (self.flat if buf is None else buf)[off:off + math.prod(shape)].view(shape)

    def cat_view(self, kind, l, buf=None):
        """[fwd; reverse] concatenation (contiguous by construction)."""
        a = self.view(f"mix.layer.{kind}_l{l}", buf)
        off = self.offsets[f"mix.layer.{kind}_l{l}"][0]
        n = a.numel()
        base = self.flat if buf is None else buf
        return base[off:off + 2 * n].view(2 * a.shape[0], *a.shape[1:]) if a.dim() == 2 else base[off:off + 2 * n]

    def bucket_split(self):
        """Index into grad_ext between the data-parallel buckets: [0, split) = the status flag and
        every recurrent layer (complete after the last BPTT), [split, end) = the Linear, the speaker
        embedding and ADDJUST (complete before the first BPTT)."""
        return 4 + self.offsets["mix.Linear.weight"][0]

    def bucket_mid(self, layer):
        """Index into grad_ext where the recurrent layers >= ``layer`` start (layers are contiguous in
        order): the three-bucket step's middle bucket is [bucket_mid(layer), bucket_split())."""
        return 4 + self.offsets[f"mix.layer.weight_ih_l{layer}"][0]

    def named_parameters(self):
        return {name: self.view(name) for name, _ in self.specs}

    def reset_parameters(self, seed=1):
        """torch default initialisers (nn.LSTM/GRU, nn.Linear, nn.Embedding)."""
        g = torch.Generator().manual_seed(seed)
        for name, shape in self.specs:
            if name.startswith("mix.layer."):
                k = 1.0 / math.sqrt(self.H)
                t = torch.empty(shape).uniform_(-k, k, generator=g)
            elif name == "emb.layer.weight":
                t = torch.randn(shape, generator=g)
            elif name.endswith("bias"):
                k = 1.0 / math.sqrt(2 * self.H)
                t = torch.empty(shape).uniform_(-k, k, generator=g)
            else:
                k = 1.0 / math.sqrt(shape[1])
                t = torch.empty(shape).uniform_(-k, k, generator=g)
            self.view(name).copy_(t)

    def load_state_dict(self, sd):
        for name, _ in self.specs:
            self.view(name).copy_(sd[name].to(torch.float32))

    def state_dict(self):
        return {name: self.view(name).detach().clone() for name, _ in self.specs}


class SepTrainer:
    """Buffers and the step schedule for one (B, K, N) workload."""

    def __init__(self, net, batch, k, n_samples, mode="label", precision="fp32", lr=2e-4, sum_weight=0.5,
                 loss_channels=None, betas=(0.9, 0.999), eps=1e-8, process_group=None, rnn_precision=None):
        if mode not in ("label", "pit", "crm"):
            raise ValueError(mode)
        if (mode == "crm") != net.crm:
            raise ValueError("cRM mode needs a cRM net (query width 2E) and vice versa")
        self.net, self.B, self.K, self.N = net, batch, k, n_samples
        self.mode, self.precision = mode, precision
        # recurrent matvec precision (defaults to the GEMM precision): "fp32" exact VALU,
        # "bf16" MFMA with fp32 accumulate and fp32 cell state
        self.rnn_precision = rnn_precision or precision
        self.lr, self.betas, self.eps = lr, betas, eps
        self.pg = process_group
        from . import dp

        # data parallel: the gradient is all-reduced with SUM and Adam applies 1 / world
        self.world = dp.world(process_group) if process_group is not None else 1
        self.T = ops.n_frames(n_samples)
        self.F = net.F
        dev = net.device
        B, K, N, T, F, H = batch, k, n_samples, self.T, net.F, net.H
        NGH = _ngate(net.cell) * H
        BT = B * T
        f32 = dict(device=dev, dtype=torch.float32)
        # mixtures and scaled sources in ONE signal buffer [B + B K, N] (magnitude modes: one STFT
        # launch over both, their magnitudes likewise adjacent)
        self._sig = torch.empty(B + B * K, N, **f32)
        self.mix = self._sig[:B]
        self.src = self._sig[B:].view(B, K, N)
        self.stats = torch.empty(32 * B * K, **f32)  # mixing partials (dl4ss_mix_sources)
        if mode == "crm":
            self.mag_mix = torch.empty(B, T, F, **f32)
            self.Xc_mix = torch.empty(B, T, F, 2, **f32)
            self.Xc_src = torch.empty(B, K, T, F, 2, **f32)
        else:
            self.Xc_mix = None
            self._mag = torch.empty(B + B * K, T, F, **f32)
            self.mag_mix = self._mag[:B]
            self.mag_src = self._mag[B:].view(B, K, T, F)
        self.out = [torch.empty(B, T, 2 * H, **f32) for _ in range(net.L)]
        self.hprev = [torch.empty(B, T, 2 * H, **f32) for _ in range(net.L)]
        self.act = [torch.empty(B, T, 2, 4 * H, **f32) for _ in range(net.L)]
        self.cs = [torch.empty(B, T, 2, H, **f32) for _ in range(net.L)] if net.cell == "lstm" else None
        self.G = torch.empty(BT, 2 * NGH, **f32)  # input projection, reused as dG
        self.dGh = torch.empty(BT, 2 * NGH, **f32) if net.cell == "gru" else None
        self.dH = [torch.empty(BT, 2 * H, **f32), torch.empty(BT, 2 * H, **f32)]
        self.V = torch.empty(BT, F * net.E, **f32)  # tanh output; overwritten in place by dPre
        W = net.W
        self.q = torch.empty(B, K, W, **f32)
        self.mean = torch.empty(B, 2 * H, **f32)
        self.dq = torch.empty(B, K, W, **f32)
        self.dh_bcast = torch.empty(B, 2 * H, **f32)
        self.nblk = _lib.query("dl4ss_attn_nblk", T, F)
        self.part_loss = torch.empty(B, self.nblk, K * K + 1, **f32)
        self.part_dq = torch.empty(B, self.nblk, K, W, **f32)
        self.perm = torch.empty(B, K, device=dev, dtype=torch.int32)
        self.loss = torch.zeros(3, **f32)
        ws = _lib.query("dl4ss_birnn_workspace_bytes", CELLS[net.cell], B, H)
        if ws < 0:
            raise RuntimeError("unsupported BiRNN configuration")
        self.ws_bytes = ws
        self.rnn_ws = torch.empty((ws + 7) // 8, device=dev, dtype=torch.int64)
        # bf16 fast path: one workspace per (layer, pass) (DL4SS_RNN_WS_ZEROED) instead of a memset
        # in front of every recurrence launch.  Zeroed once: a launch that completes leaves its
        # workspace fit for the next launch of the same shape (T >= 4: no stale tag can match, and
        # the packed kernels put their start counters / placement granules back, release_start in
        # birnn.hip), so there is no per-step fill (round 5, 10.4 us); check() zeroes it again after
        # a timed-out launch, whose half-written hand-offs could.  DL4SS_WS_FILL=1: the fill per step.
        w8 = (ws + 255) // 256 * 32
        self.rnn_ws_all = torch.zeros(2, net.L * w8, device=dev, dtype=torch.int64)  # [fwd | bwd][layer]
        self._w8 = w8
        self._ws_fill = self.T < 4 or os.environ.get("DL4SS_WS_FILL", "0") == "1"
        # {hand-off timed out, refused-update count} (the recurrence kernels set [0]; the guarded
        # Adam counts its refusals in [1])
        self.status = torch.zeros(2, device=dev, dtype=torch.int32)
        self.m = torch.zeros_like(net.flat)
        self.v = torch.zeros_like(net.flat)
        self.step_count = 0
        nch = loss_channels if loss_channels else K
        self.s1 = 1.0 / (B * nch * T * F)
        self.s2 = 0.0 if (mode == "crm" or loss_channels) else sum_weight / (B * T * F)
        self.spk = torch.empty(B, K, device=dev, dtype=torch.int32)
        # bf16 mode: every GEMM of the step runs on the hand-written LDS-DMA MFMA kernel
        # (gemm_gl.hip; deterministic split-K) and every operand is produced directly as bf16:
        # the BiRNN kernels write bf16 h / h_{t-1} / dG / dGh (and fuse the bias gradients), the
        # attention kernel writes bf16 dPre, the weights and the layer-0 features are converted
        # once per step.  Rows are padded to multiples of 8 (16-B aligned operand rows).
        # "bf16s": the bf16 step with SPLIT-precision forward GEMMs -- every forward GEMM operand as
        # hi + lo bf16 ([x_hi | x_lo | x_hi] . [w_hi | w_hi | w_lo], K' = 3 K, fp32-accurate to ~2^-16;
        # dl4ss_f32_to_bf16_hilo), V = tanh(Linear) kept fp32 -- while the recurrence (bf16 MFMA
        # matvec, fp32 state) and the whole backward stay the bf16 step's.  On the BiGRU nets (C1 / C3 /
        # C4) every bf16 forward-GEMM operand costs ~1e-3 of masked-magnitude error (tools/bf16_budget.py)
        # and the all-bf16 step misses the north-star 1e-3; this mode keeps only the recurrence's
        # rounding (~0.3e-3).
        # "bf16s2": bf16s with the split only where the error budget needs it (round 5): the input
        # projections of layers >= 1 take two terms, [x_hi | x_hi] . [w_hi | w_lo] = x_hi w (K' = 2 K:
        # the layer inputs rounded, the weights exact; tools/bf16_budget.py C4: 0.56e-3 with the
        # recurrence's rounding, vs 1.5e-3 for rounded weights), the first layer and the Linear keep
        # three.  Quoted for C4 (BiGRU-2L), whose budget allows it.
        if precision in ("bf16s", "bf16s2") and self.rnn_precision == precision:
            self.rnn_precision = "bf16"
        self.split = precision in ("bf16s", "bf16s2")
        self.split_x2 = precision == "bf16s2"
        if self.split and self.rnn_precision != "bf16":
            raise ValueError(f"precision '{precision}' runs the bf16 recurrence (rnn_precision bf16)")
        self.fast = precision in ("bf16", "bf16s", "bf16s2") and self.rnn_precision == "bf16"
        self.dh_split = int(os.environ.get("DL4SS_DH_SPLIT", "3"))  # dH split-K (tuning knob, A/B runs)
        # dH's split-K slabs summed by the top layer's BPTT as it loads dOut (DL4SS_RNN_DOUT_SLABS, round 6):
        # no combine launch between the dH GEMM and the first BPTT.  Set per trainer in the bf16 step
        # when the BPTT plan has batch chunks >= 4 (the packed loader that sums them); DL4SS_DH_SLABS=0: the
        # combine launch (A/B)
        self.dh_slabs = 1
        self.dx_split = int(os.environ.get("DL4SS_DX_SPLIT", "1"))  # dX split-K (tuning knob, A/B runs)
        # BPTT bias partials reduced once after the last BPTT instead of after each (A/B knob)
        self.defer_bias = os.environ.get("DL4SS_DEFER_BIAS", "1") != "0"
        # Forward input projections x W_ih^T + b_ih formed inside the packed recurrence kernel
        # (dl4ss_birnn_fwd_xw) instead of a gemm_gl launch + a G buffer round trip; bitwise the same
        # G (tests/test_rnn_xw_gpu.py).  Each tile's projection of a block of 16 / BC steps is one
        # MFMA chain, split one part per step over the waves with slack (birnn.hip).  DL4SS_RNN_XW:
        # "1" (default) every layer (C2, per launch: 600-wide layers 351 us vs 328 + 52 us for
        # recurrence + GEMM, first layer 313 vs 328 + 30), "l0" the first layer only, "0" none.
        xw = os.environ.get("DL4SS_RNN_XW", "1")
        if xw not in ("0", "1", "l0"):
            raise ValueError(f"DL4SS_RNN_XW={xw}: expected 0, 1 or l0")
        self.xw = self.fast and xw != "0" and not self.split
        self.xw_kmax = 160 if xw == "l0" else 640
        # bf16s: the first layer's split-operand projection ([x_hi | x_lo | x_hi] . [w_hi | w_hi | w_lo],
        # K' = 3 pad8(F) = 408 <= 640) fused into its recurrence too -- the same k-ordered chain + b_ih as
        # the split GEMM; the 600-wide layers' K' = 1800 stays a GEMM
        self.xw_split0 = self.split and xw != "0"
        # data parallel, bf16 step: the gradient leaves in two buckets ("can
        # overlap with BPTT of the lower layers").  The Linear / embedding / ADDJUST gradients are
        # complete at the end of the BPTT chain (dW_lin on the side stream beside it, or on its own
        # before it) and their all-reduce runs beside the recurrent layers' grouped weight-gradient
        # launch; the recurrent layers' bucket follows that launch.  (Round 5 first started the side
        # GEMM and the early all-reduce eagerly between two graph replays: the side GEMM then shared a
        # hardware queue with the replayed BPTT chain and ran before it, 4.91 vs 3.51 ms per step.)
        # DL4SS_DP_BUCKETS=0: one flat all-reduce after the step's backward.
        # Three buckets (round 6, DL4SS_DP_BUCKETS=3; L >= 2): the grouped weight-gradient launch is split in
        # two -- the upper layers (>= dp_layer = L // 2) first, whose all-reduce then runs beside the lower
        # layers' launch -- and only the lower layers + the status flag follow it.  Measured at world size 1
        # over RCCL (tools/dist_ab.sh, profiles/r06_dist_buckets_ab.txt): 3.61 ms per step against 3.50 for
        # two buckets and 3.48 flat -- the two half launches each pay their own ramp, tail and split-K
        # combine (+~90 us) and the third replay ~20 us, more than the ~0.03 ms of all-reduce the middle
        # bucket could hide at 8 ranks.  So the default stays "2" (round 5: one grouped
        # launch, flag + layers behind it); "0": one flat all-reduce.
        nb = os.environ.get("DL4SS_DP_BUCKETS", "2")
        if nb not in ("0", "1", "2", "3"):
            raise ValueError(f"DL4SS_DP_BUCKETS={nb}: expected 0, 2 or 3")
        self.buckets = process_group is not None and self.fast and net.L <= 5 and nb != "0"
        self.dp_layer = net.L // 2 if (self.buckets and nb == "3" and net.L >= 2) else None
        self._works = []
        self._in_chain = False
        # The Linear's weight and bias gradients on a SIDE STREAM beside the BPTT chain (round 5): the
        # persistent recurrence keeps its grid within the CUs minus 1/16 (dl4ss_birnn_plan_info), so
        # `free` CUs idle through the chain.  dW_lin (and the bias gradient as the row sums of the same
        # dPre fragments, dl4ss_gemm_bf16_gl_grouped_ex rowsum) runs there as a persistent launch of one
        # 256 x 128 three-stage workgroup per free CU, from the end of the dH GEMM to the grouped
        # launch, which it joins.  C2 (rocprofv3 r05e): the side launch takes 1.41 ms of the 1.78 ms
        # chain, the BPTTs are unchanged (406 / 399 / 396 / 397 vs 408 / 398 / 398 / 398 us), and the
        # grouped launch + combine go 336 -> 230 us.  On by a cost model (the side launch must fit in
        # the chain: dW_lin's FLOPs at ~2.75 TFLOP/s per free CU vs ~1.75 us per dependent step and
        # layer); DL4SS_SIDE_DWLIN = "0" off, "1" on, or "grid,cfg,split[,one_per_cu]" to force a shape.
        self.side = None
        self._side_stream = None
        self._side_gemm = None
        # The side launch is enqueued after the first BPTT, its fork still at the dH GEMM (an event): the
        # captured graph then keeps the chain on the main queue and puts the side GEMM on the second --
        # the first-enqueued child of the fork stays on the parent's queue.  Enqueued before the BPTT
        # the side GEMM kept it and the chain paid a cross-queue wait at the fork (11 vs 5 us) and at
        # the join (9.5 vs 6 us): 3.457-3.463 vs 3.463-3.469 ms per step (A/B x3,
        # profiles/r05_side_late_ab.txt).  DL4SS_SIDE_LATE=0 restores the early enqueue (A/B).
        self._side_late = os.environ.get("DL4SS_SIDE_LATE", "1") != "0"
        self._fork_ev = None
        side = os.environ.get("DL4SS_SIDE_DWLIN", "")
        if self.fast and net.L <= 5 and side != "0" and dev.type == "cuda":
            if side and side != "1":
                v = [int(x) for x in side.split(",")]
                self.side = (v[0], v[1], v[2], bool(v[3]) if len(v) > 3 else True)
            else:
                plan = ops.birnn_plan(net.cell, B, H)
                free = torch.cuda.get_device_properties(dev).multi_processor_count - (plan["grid"] if plan else 1 << 30)
                flops = 2.0 * (F * net.E) * (2 * H) * BT
                if free >= 8 and (flops / (free * 2.75e12) < net.L * T * 1.75e-6 * 0.85 or side == "1"):
                    self.side = (free, 2, 1, False)
        # No zeroing pass over the flat gradient (round 5): in the grouped bf16 backward every
        # gradient has exactly one writer -- the grouped / side GEMMs (beta 0), the bias reduce, the
        # Linear-bias row sums or colsum, the query backward (beta 0: it also zeroes the embedding
        # rows no speaker of the batch owns) -- and each writes its region without reading it.
        # Bitwise the zeroed form (0 + x = x).  DL4SS_GRAD_ZERO=1 restores the zeroing (A/B).
        self.zero_free = (self.fast and net.L <= 5 and self.defer_bias and
                          os.environ.get("DL4SS_GRAD_ZERO", "0") != "1")
        self._gbeta = 0.0 if self.zero_free else 1.0
        # the bf16 weight copies kept by Adam (dl4ss_adam_guarded_dp_scaled_bf16) instead of a
        # conversion launch per step; DL4SS_ADAM_SHADOW=0: the conversion every step (A/B)
        self._shadow_on = self.fast and os.environ.get("DL4SS_ADAM_SHADOW", "1") != "0"
        self._wb_ver = None
        if self.fast:
            bf = dict(device=dev, dtype=torch.bfloat16)
            p8 = lambda n: (n + 7) // 8 * 8
            self.p8 = p8
            D0 = net.F
            self.xb0 = torch.zeros(BT, p8(D0), **bf)  # (row padding zero: the STFT writes columns < F only)
            self.outb = [torch.empty(BT, p8(2 * H), **bf) for _ in range(net.L)]
            self.hprevb = [torch.empty(BT, 2 * p8(H), **bf) for _ in range(net.L)]
            # every layer's bf16 dG (and GRU dGh) stays until the end of backward: the weight
            # gradients of all layers run as one grouped GEMM launch after the last BPTT
            self.dGb_l = [torch.empty(BT, 2 * NGH, **bf) for _ in range(net.L)]
            self.dGb = self.dGb_l[0]
            # GRU dGh: each direction's gate columns start 16-B aligned (900 -> 904,
            # DL4SS_RNN_DGH_PAD8): 16-B aligned LDS-DMA operand rows for each direction's dW_hh
            self.ngh_p8 = p8(NGH)
            self.dGhb_l = [torch.empty(BT, 2 * self.ngh_p8, **bf) for _ in range(net.L)] if net.cell == "gru" else None
            self.dGhb = self.dGhb_l[0] if self.dGhb_l else None
            self._dw_group = None
            # zero row padding (never written): gemm_gl reads k-contiguous rows in 8-element chunks
            self.dPreb = torch.zeros(BT, p8(F * net.E), **bf)
            # gemm_gl split-K slabs (the largest split of _backward_fast)
            FE_ = F * net.E
            gl_need = max(_lib.query("dl4ss_gemm_bf16_gl_ws_bytes", BT, 2 * H, FE_, max(1, self.dh_split), 1),
                          _lib.query("dl4ss_gemm_bf16_gl_ws_bytes", BT, 2 * H, 2 * NGH, max(1, self.dx_split), 1),
                          _lib.query("dl4ss_gemm_bf16_gl_ws_bytes", FE_, 2 * H, BT, 2, 1),
                          _lib.query("dl4ss_gemm_bf16_gl_ws_bytes", 2 * NGH, 2 * H, BT, 4, 1),
                          _lib.query("dl4ss_gemm_bf16_gl_ws_bytes", NGH, H, BT, 8, 2))
            self.gl_ws = torch.empty(max(gl_need, 1), device=dev, dtype=torch.uint8)
            plan = ops.birnn_plan(net.cell, B, H) if dev.type == "cuda" else None
            nsl = _lib.query("dl4ss_gemm_bf16_gl_ws_bytes", BT, 2 * H, F * net.E, max(1, self.dh_split), 1) // \
                (BT * 2 * H * 4)
            # three slabs only: the BPTT's two- and four-slab instances measured 366 / 437 us per launch
            # against 308 for one or three slabs (tools/slab_probe.py, profiles/r06_slab_probe.jsonl)
            if os.environ.get("DL4SS_DH_SLABS", "1") != "0" and plan is not None and plan["BC"] == 4 and nsl == 3:
                self.dh_slabs = int(nsl)
                # the slabs' own workspace: other split-K GEMMs between dH and the BPTT (dW_lin off the side
                # stream) must not overwrite them
                self.dh_ws = torch.empty(nsl * BT * 2 * H * 4, device=dev, dtype=torch.uint8)
            # partial sums of the deterministic Linear-bias colsum (dl4ss_colsum_bf16_det)
            pb = _lib.query("dl4ss_colsum_bf16_part_bytes", BT, F * net.E)
            self.colsum_part = torch.empty(max(1, pb // 4), device=dev, dtype=torch.float32)
            # V = tanh(Linear) in bf16 (even row length); bf16s keeps V in fp32 (self.V)
            self.Vb = None if self.split else torch.empty(BT, F * net.E, **bf)
            self.wb_ih = [torch.empty(2 * NGH, p8(F if l == 0 else 2 * H), **bf) for l in range(net.L)]
            self.wb_lin = torch.empty(F * net.E, p8(2 * H), **bf)
            if self.split:  # split-precision forward operands (K' = 3 segments of pad8(K) each)
                self.seg = [p8(F if l == 0 else 2 * H) for l in range(net.L)]
                self.xs0 = torch.empty(BT, 3 * self.seg[0], **bf)
                self.xs = torch.empty(BT, 3 * p8(2 * H), **bf)
                self.ws_ih = [torch.empty(2 * NGH, 3 * self.seg[l], **bf) for l in range(net.L)]
                self.ws_lin = torch.empty(F * net.E, 3 * p8(2 * H), **bf)
            if net.cell == "lstm":  # the LSTM BPTT never reads the fp32 h_{t-1}
                self.hprev = [None] * net.L

    # ------------------------------------------------------------------ features
    def features(self, raw, gains):
        ops.mix_sources(raw, gains, out_src=self.src, out_mix=self.mix, stats_ws=self.stats)
        self._stfts()

    def _stfts(self):
        """The step's STFTs: cRM, the mixtures' complex + magnitude and the sources' complex
        spectra (two launches); magnitude modes, mixtures and sources in one launch over the
        shared signal buffer."""
        B, K, N = self.B, self.K, self.N
        # bf16 step: the mixtures' magnitudes also land in bf16 in the recurrence's input rows (xb0)
        xb = dict(out_bf16=self.xb0, n_bf16=B) if self.fast else {}
        if self.mode == "crm":
            ops.stft(self.mix, complex_out=True, mag_out=True, out_c=self.Xc_mix, out_mag=self.mag_mix, **xb)
            ops.stft(self.src.view(B * K, N), complex_out=True, mag_out=False, out_c=self.Xc_src.view(B * K, self.T,
                                                                                                     self.F, 2))
        else:
            ops.stft(self._sig, complex_out=False, mag_out=True, out_mag=self._mag, **xb)
        self._xb0_fresh = self.fast

    # ------------------------------------------------------------------ forward
    def _to_bf16_rows(self, x, out):
        """out[:, :cols] = bf16(x), zero row padding (dl4ss_f32_to_bf16_2d)."""
        _lib.call("dl4ss_f32_to_bf16_2d", _lib.ptr(x, True), x.stride(0), x.shape[0], x.shape[1], _lib.ptr(out),
                  out.stride(0), _lib.stream_ptr())

    def params_changed(self):
        """Tell the trainer that net.flat was rewritten by means that may bypass torch's version
        counter (a raw-pointer kernel, a collective, `.data`): the next step of every trainer on
        this net re-derives the bf16 weight copies instead of trusting the ones Adam keeps."""
        self.net.params_changed()
        self._wb_ver = None

    def _wb_key(self):
        return (self.net.generation, self.net.flat._version)

    def _wb_stale(self):
        return self._wb_ver is None or self._wb_ver != self._wb_key()

    def _weights_to_bf16(self, force=False):
        """The bf16 copies of every layer's W_ih and the Linear weight, one launch
        (dl4ss_f32_to_bf16_2d_multi) -- only when the parameters changed by other means than this
        trainer's Adam, which writes the copies itself (dl4ss_adam_guarded_dp_scaled_bf16, round 5):
        a torch in-place op on net.flat (a checkpoint load, the DP broadcast, a test's state restore)
        bumps its version counter, the device-side Adam does not -- it bumps the net's generation,
        so another trainer on the same net sees the change."""
        net = self.net
        if not hasattr(self, "_cvt_args"):
            pairs = [(net.cat_view("weight_ih", l), self.wb_ih[l]) for l in range(net.L)]
            pairs.append((net.view("mix.Linear.weight"), self.wb_lin))
            n = len(pairs)
            P = ctypes.c_void_p
            self._cvt_args = (n, (P * n)(*[x.data_ptr() for x, _ in pairs]),
                              (ctypes.c_longlong * n)(*[x.stride(0) for x, _ in pairs]),
                              (ctypes.c_int * n)(*[x.shape[0] for x, _ in pairs]),
                              (ctypes.c_int * n)(*[x.shape[1] for x, _ in pairs]),
                              (P * n)(*[y.data_ptr() for _, y in pairs]),
                              (ctypes.c_longlong * n)(*[y.stride(0) for _, y in pairs]))
            base = net.flat.data_ptr()
            assert all(x.is_contiguous() for x, _ in pairs)
            self._shadow = (n, (ctypes.c_longlong * n)(*[(x.data_ptr() - base) // 4 for x, _ in pairs]),
                            self._cvt_args[3], self._cvt_args[4], self._cvt_args[5], self._cvt_args[6])
        if not force and self._shadow_on and not self._wb_stale():
            return
        _lib.call("dl4ss_f32_to_bf16_2d_multi", *self._cvt_args, _lib.stream_ptr())
        self._wb_ver = self._wb_key()

    @staticmethod
    def _hilo(x, y, segw, pattern, nseg=3):
        """y = the split image of the fp32 rows x: nseg segments of segw, hi / lo by pattern bits."""
        _lib.call("dl4ss_f32_to_bf16_hilo", _lib.ptr(x, True), x.stride(0), x.shape[0], x.shape[1], _lib.ptr(y),
                  y.stride(0), segw, nseg, pattern, _lib.stream_ptr())

    def _forward_split(self, x):
        """The "bf16s" forward: each layer's input projection and the Linear as ONE gemm_gl GEMM over
        split operands [x_hi | x_lo | x_hi] . [w_hi | w_hi | w_lo] (K' = 3 K), the packed bf16
        recurrence reading G, V = tanh(Linear) in fp32.  The bf16 copies the backward uses (the
        hi weights, bf16 features, the recurrence's bf16 layer outputs) are written as in the bf16 step."""
        net, B, T, H = self.net, self.B, self.T, self.net.H
        st = _lib.stream_ptr()
        cell = CELLS[net.cell]
        A_SPLIT, W_SPLIT = 0b010, 0b100  # [hi | lo | hi] and [hi | hi | lo]
        if self._ws_fill:
            self.rnn_ws_all.zero_()  # every layer's forward AND BPTT hand-off workspaces, one fill per step
        self._weights_to_bf16()
        A2, W2 = 0b00, 0b10  # bf16s2, layers >= 1: [hi | hi] and [hi | lo]
        for l in range(net.L):
            if l >= 1 and self.split_x2:
                self._hilo(net.cat_view("weight_ih", l), self.ws_ih[l], self.seg[l], W2, 2)
            else:
                self._hilo(net.cat_view("weight_ih", l), self.ws_ih[l], self.seg[l], W_SPLIT)
        self._hilo(net.view("mix.Linear.weight"), self.ws_lin, self.p8(2 * H), W_SPLIT)
        if not self._xb0_ok:
            self._to_bf16_rows(x, self.xb0)
        self._mean_done = False
        self._hilo(x, self.xs0, self.seg[0], A_SPLIT)
        xin = self.xs0
        for l in range(net.L):
            Ks = xin.shape[1]
            if (l == 0 and self.xw_split0 and
                    _lib.query("dl4ss_birnn_fwd_xw_supported", cell, B, T, H, Ks) == 1):
                wih = self.ws_ih[0]
                _lib.call("dl4ss_birnn_fwd_xw_ex", cell, B, T, H, _lib.ptr(xin), Ks, xin.stride(0), _lib.ptr(wih),
                          wih.stride(0), _lib.ptr(net.cat_view("bias_ih", 0)),
                          _lib.ptr(net.cat_view("weight_hh", 0)), _lib.ptr(net.cat_view("bias_hh", 0)),
                          _lib.ptr(self.out[0]), _lib.ptr(self.hprev[0]), _lib.ptr(self.act[0]),
                          _lib.ptr(self.cs[0]) if self.cs else None, _lib.ptr(self.outb[0]), _lib.ptr(self.hprevb[0]),
                          None, _lib.ptr(self._ws_slot(0, False)), self.ws_bytes, _lib.ptr(self.status), st, 1)
                xin = self._split_input(0)
                continue
            self._gemm_fwd(xin, self.ws_ih[l][:, :xin.shape[1]], net.cat_view("bias_ih", l), self.G)
            _lib.call("dl4ss_birnn_fwd_ex", cell, 1 | WS_ZEROED, B, T, H, _lib.ptr(self.G),
                      _lib.ptr(net.cat_view("weight_hh", l)), _lib.ptr(net.cat_view("bias_hh", l)),
                      _lib.ptr(self.out[l]), _lib.ptr(self.hprev[l]), _lib.ptr(self.act[l]),
                      _lib.ptr(self.cs[l]) if self.cs else None, _lib.ptr(self.outb[l]), _lib.ptr(self.hprevb[l]),
                      _lib.ptr(self._ws_slot(l, False)), self.ws_bytes, _lib.ptr(self.status), st)
            xin = self._split_input(l)
        self._gemm_fwd(xin, self.ws_lin, net.view("mix.Linear.bias"), self.V, ops.EPI_TANH)

    def _split_input(self, l):
        """Layer l's output as the split A image of the next GEMM: [hi | lo | hi] (three terms), or
        [hi | hi] (bf16s2, into layers >= 1: two terms, K' = 2 pad8(2H)); the Linear's is three."""
        H, w = self.net.H, self.p8(2 * self.net.H)
        src = self.out[l].view(self.B * self.T, 2 * H)
        if self.split_x2 and l < self.net.L - 1:
            self._hilo(src, self.xs, w, 0b00, 2)
            return self.xs[:, :2 * w]
        self._hilo(src, self.xs, w, 0b010)  # A_SPLIT
        return self.xs

    def _forward_fast(self, x):
        net, B, T, H = self.net, self.B, self.T, self.net.H
        BT = B * T
        st = _lib.stream_ptr()
        cell = CELLS[net.cell]
        if self._ws_fill:
            self.rnn_ws_all.zero_()  # every layer's forward AND BPTT hand-off workspaces, one fill per step
        self._weights_to_bf16()
        if not self._xb0_ok:
            self._to_bf16_rows(x, self.xb0)
        xb = self.xb0[:, :x.shape[1]]
        self._mean_done = False
        for l in range(net.L):
            D = xb.shape[1]
            hp = self.hprev[l]
            if self.xw and D <= self.xw_kmax and _lib.query("dl4ss_birnn_fwd_xw_supported", cell, B, T, H, D) == 1:
                wih = self.wb_ih[l]
                # no fp32 layer output (the next layer and the GEMMs read the bf16 one); the last layer
                # forms the time mean of ADDJUST / the query inside the recurrence (h_mean)
                last = l == net.L - 1
                _lib.call("dl4ss_birnn_fwd_xw_ex", cell, B, T, H, _lib.ptr(xb, strided=True), D, xb.stride(0),
                          _lib.ptr(wih), wih.stride(0), _lib.ptr(net.cat_view("bias_ih", l)),
                          _lib.ptr(net.cat_view("weight_hh", l)), _lib.ptr(net.cat_view("bias_hh", l)),
                          None, _lib.ptr(hp), _lib.ptr(self.act[l]),
                          _lib.ptr(self.cs[l]) if self.cs else None, _lib.ptr(self.outb[l]), _lib.ptr(self.hprevb[l]),
                          _lib.ptr(self.mean) if last else None,
                          _lib.ptr(self._ws_slot(l, False)), self.ws_bytes, _lib.ptr(self.status), st, 1)
                self._mean_done = last
                xb = self.outb[l][:, :2 * H]
                continue
            self._gemm_fwd(xb, self.wb_ih[l][:, :D], net.cat_view("bias_ih", l), self.G)
            last = l == net.L - 1  # (the time mean formed as on the fused path)
            _lib.call("dl4ss_birnn_fwd_mean", cell, 1 | WS_ZEROED, B, T, H, _lib.ptr(self.G),
                      _lib.ptr(net.cat_view("weight_hh", l)), _lib.ptr(net.cat_view("bias_hh", l)),
                      _lib.ptr(self.out[l]), _lib.ptr(hp), _lib.ptr(self.act[l]),
                      _lib.ptr(self.cs[l]) if self.cs else None, _lib.ptr(self.outb[l]), _lib.ptr(self.hprevb[l]),
                      _lib.ptr(self.mean) if last else None,
                      _lib.ptr(self._ws_slot(l, False)), self.ws_bytes, _lib.ptr(self.status), st)
            self._mean_done = last
            xb = self.outb[l][:, :2 * H]
        self._gemm_fwd(xb, self.wb_lin[:, :2 * H], net.view("mix.Linear.bias"), self.Vb, ops.EPI_TANH_BF16)

    def _gemm_fwd(self, x, w, bias, out, epilogue=ops.EPI_NONE):
        """out = x w^T + bias (epilogue): the input projections and the Linear (+ tanh -> bf16 V)"""
        ops.gemm_bf16_gl(x, w, transB=True, bias=bias, epilogue=epilogue, out=out)

    def forward(self, feats=None):
        net, B, T, H = self.net, self.B, self.T, self.net.H
        BT = B * T
        x = (self.mag_mix if feats is None else feats).reshape(BT, -1)
        # the STFT of this step already wrote x's bf16 rows (self.xb0) unless the features came from elsewhere
        self._xb0_ok = feats is None and getattr(self, "_xb0_fresh", False)
        self._xb0_fresh = False
        st = _lib.stream_ptr()
        cell = CELLS[net.cell]
        if self.fast:
            if self.split:
                self._forward_split(x)
            else:
                self._forward_fast(x)
            wadj = net.view("adj.layer.weight") if net.adjust else None
            h_last = None if (not self.split and self._mean_done) else _lib.ptr(self.out[-1])
            _lib.call("dl4ss_query_fwd", h_last, B, T, 2 * H, _lib.ptr(self.spk),
                      _lib.ptr(net.view("emb.layer.weight")), _lib.ptr(wadj), self.K, net.W, _lib.ptr(self.q),
                      _lib.ptr(self.mean), st)
            self._feats = x
            return
        for l in range(net.L):
            ops.gemm(x, net.cat_view("weight_ih", l), transB=True, bias=net.cat_view("bias_ih", l), out=self.G,
                     precision=self.precision)
            _lib.call("dl4ss_birnn_fwd", cell, ops.PREC[self.rnn_precision], B, T, H, _lib.ptr(self.G),
                      _lib.ptr(net.cat_view("weight_hh", l)), _lib.ptr(net.cat_view("bias_hh", l)),
                      _lib.ptr(self.out[l]), _lib.ptr(self.hprev[l]), _lib.ptr(self.act[l]), _lib.ptr(self.cs[l]) if self.cs else None, _lib.ptr(self.rnn_ws),
                      self.ws_bytes, _lib.ptr(self.status), st)
            x = self.out[l].view(BT, 2 * H)
        ops.gemm(x, net.view("mix.Linear.weight"), transB=True, bias=net.view("mix.Linear.bias"),
                 epilogue=ops.EPI_TANH, out=self.V, precision=self.precision)
        wadj = net.view("adj.layer.weight") if net.adjust else None
        _lib.call("dl4ss_query_fwd", _lib.ptr(self.out[-1]), B, T, 2 * H, _lib.ptr(self.spk),
                  _lib.ptr(net.view("emb.layer.weight")), _lib.ptr(wadj), self.K, net.W, _lib.ptr(self.q),
                  _lib.ptr(self.mean), st)

    def _attn_args(self):
        B, K, T, F = self.B, self.K, self.T, self.F
        TF = T * F
        if self.mode == "crm":
            return self.Xc_mix, TF, self.Xc_src, K * TF, TF
        return self.mag_mix, TF, self.mag_src, K * TF, TF

    def attn(self, pass_, perm=None, mask_out=None, pred_out=None):
        X, xs, Y, ys, yks = self._attn_args()
        grad = pass_ == 1
        dpre = _lib.ptr(self.V) if grad and not self.fast else None
        # (the COST pass gets dPre_bf16 too: it selects the same attention kernel as the GRAD pass)
        dpreb = _lib.ptr(self.dPreb) if self.fast else None
        # bf16 path: V itself is bf16 (the Linear's EPI_TANH_BF16 epilogue); bf16s: fp32 V, bf16 dPre
        bf16v = self.fast and not self.split
        fn, v = ("dl4ss_mask_attn_loss_bf16v", self.Vb) if bf16v else ("dl4ss_mask_attn_loss_ex", self.V)
        _lib.call(fn, pass_, int(self.mode == "crm"), self.B, self.K, self.T, self.F,
                  self.net.E, _lib.ptr(v), _lib.ptr(self.q), _lib.ptr(X), xs, _lib.ptr(Y), ys, yks,
                  _lib.ptr(perm), self.s1, self.s2, dpre, dpreb, self.dPreb.stride(0) if self.fast else 0,
                  _lib.ptr(self.part_loss), _lib.ptr(self.part_dq) if grad else None, _lib.ptr(mask_out),
                  _lib.ptr(pred_out), _lib.stream_ptr())

    def loss_and_grad(self):
        """Fused attention + loss + dPre (in place over V) + dq; returns loss (device)."""
        st = _lib.stream_ptr()
        perm = None
        if self.mode == "pit":
            self.attn(0)
            _lib.call("dl4ss_pit_select", _lib.ptr(self.part_loss), self.B, self.K, self.nblk, _lib.ptr(self.perm), st)
            perm = self.perm
        self.attn(1, perm)
        _lib.call("dl4ss_loss_finalize", _lib.ptr(self.part_loss), self.B, self.K, self.nblk, _lib.ptr(perm),
                  self.s1, self.s2, _lib.ptr(self.loss), _lib.ptr(self.part_dq), self.net.W, _lib.ptr(self.dq), st)
        return self.loss

    # ------------------------------------------------------------------ backward
    def _weight_grad_group(self):
        """The step's weight gradients (dW_lin, then every layer's dW_ih and both directions'
        dW_hh) as one grouped gemm_gl launch + one split-K combine (ops.GroupedGemm), after the last
        BPTT: one at a time they under-fill the chip (dW_ih 95 tiles x 4 splits, dW_hh 2 x 30 tiles
        x 8 splits, each with its own ramp and tail).  Each gradient is bitwise what a single
        launch with the same split factor produces (tests/test_gemm_grouped_gpu.py).  The weight gradients
        accumulate (beta 1) onto the zeroed flat gradient: the reference's loss.backward()
        (TDAA_beta/main_run_sstune_EvalVer.py:673).  Returns the list of launches: one, or with three
        data-parallel buckets two -- the layers >= dp_layer, then the rest -- each gradient bitwise the
        one-launch form's (same split factors)."""
        if self._dw_group is not None:
            return self._dw_group
        net, H = self.net, self.net.H
        NGH = _ngate(net.cell) * H
        FE = self.F * net.E
        g = net.grad
        hp8 = self.p8(H)
        gru = self.dGhb_l is not None
        ldgh = self.ngh_p8 if gru else NGH
        # split-K factors of the grouped launch (C2 bench, 20 steps, r03_dwg: dW_lin / dW_ih / dW_hh
        # 2/4/8 -> 4.434 ms per step, 2/4/4 4.424, 2/3/6 4.420, 1/2/4 4.405, 2/2/4 4.400): fewer, longer
        # k-ranges than the single launches wanted, and smaller slabs for the combine.  Round 4 (n-fastest
        # tiles per XCD, alternating A/B runs, profiles/r04_dw_splits.jsonl): at C2 2/1/4 3.856 ms vs
        # 2/2/4 3.869, 2/1/3 3.858, 1/2/4 3.855-3.860, 2/2/8 3.867-3.877, 2/2/2 3.880, 1/1/4 3.888; the
        # 2-layer BiGRU configs want dW_ih split (C4 2.52 vs 2.59 ms, C3 2.13 vs 2.17 ms with 2/2/4).  So
        # dW_ih goes unsplit when the group fills >= 3 waves of the 512 workgroup slots without it
        # (C2: 1793 workgroups; the BiGRU-2L nets: 999)
        def tiles(m, n):
            return ((m + 127) // 128) * ((n + 127) // 128)

        s_lin, s_hh = 2, 4
        wg1 = s_lin * tiles(FE, 2 * H) + sum(tiles(NGH * 2, self.F if l == 0 else 2 * H) for l in range(net.L)) + \
            s_hh * 2 * net.L * tiles(NGH, H)
        s_ih = 1 if wg1 >= 3 * 512 else 2
        if os.environ.get("DL4SS_DW_SPLITS"):  # A/B knob: "lin,ih,hh"
            s_lin, s_ih, s_hh = (int(v) for v in os.environ["DL4SS_DW_SPLITS"].split(","))
        self.dw_splits = (s_lin, s_ih, s_hh)

        def layer_probs(layers):
            # longest k-ranges first (dW_lin 63 k-tiles per workgroup, dW_ih 32, dW_hh 16): the short
            # ones fill the tail
            probs = []
            for l in layers:
                xb = self.xb0[:, :self.F] if l == 0 else self.outb[l - 1][:, :2 * H]
                probs.append(dict(A=self.dGb_l[l], B=xb, out=net.cat_view("weight_ih", l, g), transA=True,
                                  transB=False, beta=self._gbeta, splitk=s_ih))
            for l in layers:
                src = self.dGhb_l[l] if gru else self.dGb_l[l]
                whh = net.cat_view("weight_hh", l, g)
                for d in range(2):
                    probs.append(dict(A=src[:, d * ldgh:d * ldgh + NGH], B=self.hprevb[l][:, d * hp8:d * hp8 + H],
                                      out=whh[d * NGH:(d + 1) * NGH], transA=True, transB=False, beta=self._gbeta,
                                      splitk=s_hh))
            return probs

        lin = [] if (self.buckets or self.side) else [dict(A=self.dPreb[:, :FE], B=self.outb[-1][:, :2 * H],
                                             out=net.view("mix.Linear.weight", g), transA=True, transB=False,
                                             beta=self._gbeta, splitk=s_lin)]
        # DL4SS_DW_CFG (A/B knob): the grouped launch's tile configuration (1: 128 x 128, two workgroups
        # per CU; 2: 256 x 128 three-stage, one per CU)
        cfg = int(os.environ.get("DL4SS_DW_CFG", "1"))
        if self.dp_layer is not None:
            Ls = self.dp_layer
            self._dw_group = [ops.GroupedGemm(lin + layer_probs(range(net.L - 1, Ls - 1, -1)), net.device, cfg=cfg),
                              ops.GroupedGemm(layer_probs(range(Ls - 1, -1, -1)), net.device, cfg=cfg)]
        else:
            self._dw_group = [ops.GroupedGemm(lin + layer_probs(range(net.L - 1, -1, -1)), net.device, cfg=cfg)]
        return self._dw_group

    def _backward_fast_early(self):
        """The bf16 backward up to the first BPTT: the Linear's input gradient dH (all the BPTT chain
        waits on), its bias gradient, and -- ungrouped or data-parallel bucketed -- its weight
        gradient."""
        net, B, T, H = self.net, self.B, self.T, self.net.H
        BT = B * T
        FE = self.F * net.E
        g = net.grad
        dPreb = self.dPreb[:, :FE]
        st = _lib.stream_ptr()
        grouped = net.L <= 5  # <= 16 problems per grouped launch
        # gemm_gl split-K factors, measured per shape at C2 (tools/gemm_gl_bench.py --sweep): dH
        # 8032x600x6450 -> 3, dW_lin 6450x600x8032 -> 2, dX 8032x600x2400 -> 1, dW_ih
        # 2400x600x8032 -> 4, dW_hh 2 x 1200x300x8032 -> 8 (slabs + a fixed-order reduce)
        if self.dh_slabs > 1:  # the slabs stay in dh_ws: the top layer's BPTT sums them (DL4SS_RNN_DOUT_SLABS)
            ops.gemm_bf16_gl(dPreb, self.wb_lin[:, :2 * H], out=self.dH[0], splitk=self.dh_split, ws=self.dh_ws,
                             epilogue=ops.EPI_SPLIT_SLABS)
        else:
            ops.gemm_bf16_gl(dPreb, self.wb_lin[:, :2 * H], out=self.dH[0], splitk=self.dh_split, ws=self.gl_ws)
        if (not grouped or self.buckets) and not self.side:  # (bitwise the grouped launch's dW_lin at the same split)
            ops.gemm_bf16_gl(dPreb, self.outb[-1][:, :2 * H], transA=True, out=net.view("mix.Linear.weight", g),
                             beta=self._gbeta, splitk=2, ws=self.gl_ws)
        if not self.side:
            _lib.call("dl4ss_colsum_bf16_det_ex", _lib.ptr(self.dPreb), self.dPreb.stride(0), BT, FE,
                      _lib.ptr(net.view("mix.Linear.bias", g)), _lib.ptr(self.colsum_part),
                      self.colsum_part.numel() * 4, self._gbeta, st)
        elif self._side_late:
            if self._fork_ev is None:
                self._fork_ev = torch.cuda.Event()
            self._fork_ev.record()  # the fork point; the side launch follows the first BPTT
        else:
            self._side_launch()

    def _side_launch(self):
        """Fork: the side stream waits for the work enqueued so far on the current stream (the dH
        GEMM last), then runs the persistent dW_lin (+ bias row sums) launch beside the BPTT chain.
        Measured alternatives (tools/ab_bench.sh, C2, round 5): moving the gradient zeroing and the
        query backward onto the side stream too (beside the dH GEMM, the chain waiting on an event
        for dh_bcast) made the two BPTTs that ran beside the side GEMM take twice as long (665 vs
        338 us per launch; step 4.11 vs 3.51 ms), with or without a delay before the side GEMM and
        with the recurrence's groups formed by placement (group_pk) -- so they stay on the main
        stream, before dH."""
        net, B, T, H = self.net, self.B, self.T, self.net.H
        g = net.grad
        FE = self.F * net.E
        if self._side_stream is None:
            grid, cfg, split, one = self.side
            self._side_stream = torch.cuda.Stream(device=net.device)
            self._side_gemm = ops.GroupedGemm(
                [dict(A=self.dPreb[:, :FE], B=self.outb[-1][:, :2 * H], out=net.view("mix.Linear.weight", g),
                      transA=True, transB=False, beta=self._gbeta, splitk=split,
                      rowsum=net.view("mix.Linear.bias", g) if split == 1 else None)],
                net.device, grid=grid, cfg=cfg, one_per_cu=one)
        if self._side_late:
            self._side_stream.wait_event(self._fork_ev)
        else:
            self._side_stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self._side_stream):
            if self.side[2] != 1:  # split dW_lin: no row sums, the bias gradient by colsum
                _lib.call("dl4ss_colsum_bf16_det_ex", _lib.ptr(self.dPreb), self.dPreb.stride(0), B * T, FE,
                          _lib.ptr(net.view("mix.Linear.bias", g)), _lib.ptr(self.colsum_part),
                          self.colsum_part.numel() * 4, self._gbeta, _lib.stream_ptr())
            self._side_gemm.run()

    def _side_join(self):
        """Join: the current stream waits for the side stream's work."""
        torch.cuda.current_stream().wait_stream(self._side_stream)

    def _backward_fast(self, part="all"):
        """The bf16 backward from the first BPTT on: the BPTT / dX chain down the layers (part
        "chain", the side stream joined at its end), then the bias reduce and the grouped
        weight-gradient launch (part "wgrad")."""
        if part in ("wgrad", "upper", "lower"):
            return self._backward_wgrad("all" if part == "wgrad" else part)
        self._in_chain = True
        try:
            self._backward_chain()
        finally:
            self._in_chain = False
        if part == "all":
            self._backward_wgrad()

    def _backward_chain(self):
        """The BPTT / dX chain down the layers, the side stream joined at its end."""
        net, B, T, H = self.net, self.B, self.T, self.net.H
        BT = B * T
        NGH = _ngate(net.cell) * H
        g = net.grad
        cell = CELLS[net.cell]
        st = _lib.stream_ptr()
        gru = self.dGhb_l is not None
        grouped = net.L <= 5  # <= 16 problems per grouped launch
        dwg = self._weight_grad_group() if grouped else None
        # (the BPTT hand-off workspaces were zeroed with the forward's, in the step's one fill)
        dH = self.dH[0]
        hp8 = self.p8(H)
        ldgh = self.ngh_p8 if gru else NGH  # dW_hh operand: direction d at column d * ldgh
        for l in range(net.L - 1, -1, -1):
            dGb = self.dGb_l[l]
            dGhb = self.dGhb_l[l] if gru else dGb
            # the top layer reads dH as the dH GEMM's split-K slabs (summed as it loads them)
            slabs = self.dh_slabs if l == net.L - 1 else 1
            _lib.call("dl4ss_birnn_bwd_ex", cell, 1 | WS_ZEROED | (DEFER_BIAS if self.defer_bias else 0) |
                      (DGH_PAD8 if gru else 0) | DOUT_SLABS(slabs), B, T, H,
                      _lib.ptr(self.dh_ws) if slabs > 1 else _lib.ptr(dH),
                      _lib.ptr(self.dh_bcast) if (l == net.L - 1 and net.adjust) else None,
                      _lib.ptr(net.cat_view("weight_hh", l)), _lib.ptr(self.act[l]),
                      _lib.ptr(self.cs[l]) if self.cs else None, _lib.ptr(self.hprev[l]), None, None,
                      _lib.ptr(dGb), _lib.ptr(dGhb) if gru else None, _lib.ptr(net.cat_view("bias_ih", l, g)),
                      _lib.ptr(net.cat_view("bias_hh", l, g)), _lib.ptr(self._ws_slot(l, True)), self.ws_bytes,
                      _lib.ptr(self.status), st)
            if self.side and self._side_late and l == net.L - 1:
                self._side_launch()
            if l > 0:  # the input gradient: all the next BPTT waits on
                dH_next = self.dH[1] if dH is self.dH[0] else self.dH[0]
                ops.gemm_bf16_gl(dGb, self.wb_ih[l][:, :2 * H], out=dH_next, splitk=self.dx_split, ws=self.gl_ws)
            if not grouped:
                xb = self.xb0[:, :self.F] if l == 0 else self.outb[l - 1][:, :2 * H]
                ops.gemm_bf16_gl(dGb, xb, transA=True, out=net.cat_view("weight_ih", l, g), beta=1.0, splitk=4,
                                 ws=self.gl_ws)
                # both directions' dW_hh in one launch: member d = columns d*ldgh of dGh, d*pad8(H) of h_{t-1}
                ops.gemm_bf16_gl(dGhb[:, :NGH], self.hprevb[l][:, :H], transA=True,
                                 out=net.cat_view("weight_hh", l, g)[:NGH], beta=1.0, splitk=8, batch=2, strideA=ldgh,
                                 strideB=hp8, strideC=NGH * H, M=NGH, N=H, K=BT, ws=self.gl_ws)
            if l > 0:
                dH = dH_next
        # the side stream joins at the end of the chain (it ends inside the last BPTT): a join after the
        # grouped launch cost ~9 us more per step (the cross-queue wait in front of Adam; A/B x3, round 5)
        if self.side:
            self._side_join()

    def _backward_wgrad(self, which="all"):
        """The recurrent layers' bias reduce and grouped weight-gradient launch(es) (after the chain).
        Three data-parallel buckets: "upper" (the bias reduce + the layers >= dp_layer) and "lower"."""
        if which != "lower" and self.defer_bias:
            self._bias_reduce()
        if self.net.L <= 5:
            groups = self._weight_grad_group()
            run = groups if which == "all" else groups[:1] if which == "upper" else groups[1:]
            for grp in run:
                grp.run()

    def _bias_reduce(self):
        """Every layer's BPTT bias partials (DL4SS_RNN_DEFER_BIAS) into db_ih / db_hh, one launch."""
        net, g = self.net, self.net.grad
        if not hasattr(self, "_bias_args"):
            n = net.L
            P = ctypes.c_void_p
            self._bias_args = (n, (P * n)(*[self._ws_slot(l, True).data_ptr() for l in range(n)]),
                               (P * n)(*[net.cat_view("bias_ih", l, g).data_ptr() for l in range(n)]),
                               (P * n)(*[net.cat_view("bias_hh", l, g).data_ptr() for l in range(n)]))
        _lib.call("dl4ss_birnn_bias_reduce_ex", CELLS[net.cell], self.B, net.H, *self._bias_args, self._gbeta,
                  _lib.stream_ptr())

    def backward(self):
        self.backward_early()
        self.backward_late()

    def backward_early(self):
        """The backward up to the first BPTT: the query / embedding / ADDJUST gradients and the
        Linear's.  Every gradient of the data-parallel early bucket (the flat range from
        SepNet.bucket_split on) is complete when this returns (in stream order)."""
        net, B, T, H = self.net, self.B, self.T, self.net.H
        BT = B * T
        g = net.grad
        if not self.zero_free:
            g.zero_()
        self._query_bwd()
        if self.fast:
            self._backward_fast_early()
            return
        dPre = self.V
        hL = self.out[-1].view(BT, 2 * H)
        # grads were zeroed above: weight gradients accumulate (beta 1) with split-K
        ops.gemm(dPre, hL, transA=True, out=net.view("mix.Linear.weight", g), beta=1.0, splitk="auto",
                 precision=self.precision)
        ops.colsum(dPre, net.view("mix.Linear.bias", g))
        ops.gemm(dPre, net.view("mix.Linear.weight"), out=self.dH[0], splitk="auto", precision=self.precision)

    def _query_bwd(self):
        """SPEECH_EMBEDDING / ADDJUST backward: the embedding and ADDJUST gradients (added into the
        zeroed flat gradient, or written over it when zero_free) and dh_bcast, ADDJUST's share of the
        last layer's output gradient."""
        net, B, T, H = self.net, self.B, self.T, self.net.H
        g = net.grad
        wadj = net.view("adj.layer.weight") if net.adjust else None
        _lib.call("dl4ss_query_bwd_ex", _lib.ptr(self.dq), B, T, 2 * H, _lib.ptr(self.spk),
                  _lib.ptr(net.view("emb.layer.weight")), _lib.ptr(wadj), _lib.ptr(self.mean), self.K, net.W,
                  _lib.ptr(net.view("emb.layer.weight", g)),
                  _lib.ptr(net.view("adj.layer.weight", g)) if net.adjust else None,
                  _lib.ptr(self.dh_bcast) if net.adjust else None, net.num_labels, self._gbeta, _lib.stream_ptr())

    def backward_late(self):
        """The BPTT chain and the recurrent layers' weight / bias gradients, then the status flag."""
        net, B, T, H = self.net, self.B, self.T, self.net.H
        BT = B * T
        NGH = _ngate(net.cell) * H
        g = net.grad
        st = _lib.stream_ptr()
        cell = CELLS[net.cell]
        if self.fast:
            self._backward_fast()
            self._status_flag()
            return
        dH = self.dH[0]
        for l in range(net.L - 1, -1, -1):
            dG = self.G
            dGh = self.dGh if self.dGh is not None else dG
            _lib.call("dl4ss_birnn_bwd", cell, ops.PREC[self.rnn_precision], B, T, H, _lib.ptr(dH),
                      _lib.ptr(self.dh_bcast) if (l == net.L - 1 and net.adjust) else None,
                      _lib.ptr(net.cat_view("weight_hh", l)), _lib.ptr(self.act[l]),
                      _lib.ptr(self.cs[l]) if self.cs else None, _lib.ptr(self.hprev[l]), _lib.ptr(dG),
                      _lib.ptr(self.dGh) if self.dGh is not None else None, _lib.ptr(self.rnn_ws), self.ws_bytes,
                      _lib.ptr(self.status), st)
            xl = self.mag_mix.view(BT, -1) if l == 0 else self.out[l - 1].view(BT, 2 * H)
            ops.gemm(dG, xl, transA=True, out=net.cat_view("weight_ih", l, g), splitk="auto", beta=1.0,
                     precision=self.precision)
            ops.colsum(dG, net.cat_view("bias_ih", l, g))
            whh_g = net.cat_view("weight_hh", l, g)
            hp = self.hprev[l].view(BT, 2 * H)
            for d in range(2):
                ops.gemm(dGh[:, d * NGH:(d + 1) * NGH], hp[:, d * H:(d + 1) * H], transA=True,
                         out=whh_g[d * NGH:(d + 1) * NGH], splitk="auto", beta=1.0, precision=self.precision)
            ops.colsum(dGh, net.cat_view("bias_hh", l, g))
            if l > 0:
                dH_next = self.dH[1] if dH is self.dH[0] else self.dH[0]
                ops.gemm(dG, net.cat_view("weight_ih", l), out=dH_next, splitk="auto", precision=self.precision)
                dH = dH_next
        self._status_flag()

    def _status_flag(self):
        """Data parallel: this rank's hand-off status as the float behind the flat gradient
        (rewritten every step), combined by the all-reduce (allreduce()).  Without a process
        group the slot stays zero."""
        if self.pg is not None:
            _lib.call("dl4ss_status_flag", _lib.ptr(self.status), _lib.ptr(self.net.dp_flag), _lib.stream_ptr())

    def allreduce(self):
        """START the RCCL all-reduce (SUM) of the whole flat gradient, asynchronously; Adam applies
        the 1 / world of the mean (no separate pass over the buffer).  The slot in front of the
        gradient carries this rank's hand-off status flag (dl4ss_status_flag, written at the end of
        backward()): after the sum it is non-zero on every rank iff a hand-off timed out on any
        rank, and the guarded Adam reads it (a timed-out rank's incomplete gradient must
        not reach the healthy ranks' weights either).  Bucketed steps (self.buckets) use
        allreduce_early / _late.

        Contract: net.grad is complete only after wait_allreduce() (optimizer_step()
        calls it), and it then holds the SUM over ranks, not the mean -- grad_mean() is the mean."""
        if self.pg is None:
            return
        from . import dp

        self._no_collective_in_chain()
        self._works.append(dp.allreduce_sum_async(self.net.grad_ext, self.pg))

    def _no_collective_in_chain(self):
        """Invariant: no collective starts while the BPTT chain is being enqueued.  The
        persistent recurrence needs all its workgroups co-resident, and the side-stream dW_lin holds
        every CU the recurrence plan leaves free for the whole chain; a collective kernel placed
        beside the chain could keep a recurrence workgroup off the device (a hand-off timeout, then a
        refused step).  Every all-reduce of the step therefore starts after the chain."""
        if self._in_chain:
            raise RuntimeError("a gradient all-reduce was started inside the BPTT chain")

    def allreduce_early(self):
        """Start the SUM all-reduce of the early bucket (Linear, embedding, ADDJUST gradients):
        asynchronous, on the process group's stream after the work enqueued so far, beside the
        BPTT chain that follows."""
        from . import dp

        self._no_collective_in_chain()
        self._works.append(dp.allreduce_sum_async(self.net.grad_ext[self.net.bucket_split():], self.pg))

    def _early_bucket(self):
        """Bucketed data parallel: the early bucket's all-reduce (Linear -- formed on the side stream,
        joined at the end of the chain --, embedding, ADDJUST), started after the BPTT chain and
        running beside the recurrent layers' weight-gradient launch."""
        self.allreduce_early()

    def allreduce_mid(self):
        """Three buckets: start the SUM all-reduce of the upper recurrent layers (>= dp_layer), complete
        after the first weight-gradient launch, beside the second."""
        from . import dp

        self._no_collective_in_chain()
        net = self.net
        self._works.append(dp.allreduce_sum_async(net.grad_ext[net.bucket_mid(self.dp_layer):net.bucket_split()],
                                                  self.pg))

    def allreduce_late(self):
        """Start the SUM all-reduce of the late bucket: the status flag and every recurrent layer (two
        buckets), or the layers below dp_layer (three)."""
        from . import dp

        self._no_collective_in_chain()
        end = self.net.bucket_mid(self.dp_layer) if self.dp_layer is not None else self.net.bucket_split()
        self._works.append(dp.allreduce_sum_async(self.net.grad_ext[:end], self.pg))

    def wait_allreduce(self):
        """The current stream waits for every all-reduce started this step: net.grad then holds the
        gradient SUM over ranks (for callers that inspect or clip it before optimizer_step(), which
        calls this itself; grad_mean() gives the mean)."""
        for w in self._works:
            if w is not None:
                w.wait()
        self._works = []

    _wait_allreduce = wait_allreduce

    def grad_mean(self):
        """The global-batch mean gradient (a new tensor): the all-reduced SUM x 1 / world, the
        arithmetic the guarded Adam applies (gscale)."""
        self.wait_allreduce()
        return self.net.grad * (1.0 / self.world)

    def optimizer_step(self):
        """Adam on device; refused (parameters untouched, loss[0] = NaN) when a recurrence
        hand-off of this step timed out on this rank or (data parallel) on any rank -- a
        timed-out step never reaches the weights.  A refused step is counted on device
        (status[1]); check() takes the refused steps back out of step_count, so the bias
        corrections follow the updates actually applied, as torch.optim.Adam's do.  Data
        parallel: the gradient is the SUM over ranks, scaled by 1 / world inside the update."""
        self._wait_allreduce()
        self.step_count += 1
        shadow = self._shadow if (self._shadow_on and hasattr(self, "_shadow")) else None
        ops.adam_(self.net.flat, self.net.grad, self.m, self.v, self.step_count, self.lr, self.betas, self.eps,
                  status=self.status, loss=self.loss, dp_flag=self.net.dp_flag, gscale=1.0 / self.world,
                  shadow=shadow)
        # the update bypasses torch's version counter: a new generation of the parameters, whose bf16
        # copies only this trainer holds (written by the same launch), and only if they were current
        # before it -- copies stale before the update stay stale after it
        fresh = shadow is not None and not self._wb_stale()
        self.net.params_changed()
        self._wb_ver = self._wb_key() if fresh else None

    def step(self, raw, gains, spk_idx):
        """One full training step on device-resident inputs; returns the loss tensor (not synced)."""
        self.spk.copy_(spk_idx)
        self.features(raw, gains)
        self.forward()
        loss = self.loss_and_grad()
        if self.buckets:
            self.backward_early()
            self._backward_fast("chain")
            self._early_bucket()
            if self.dp_layer is not None:
                self._backward_fast("upper")
                self.allreduce_mid()
                self._backward_fast("lower")
            else:
                self._backward_fast("wgrad")
            self._status_flag()
            self.allreduce_late()
        else:
            self.backward()
            self.allreduce()
        self.optimizer_step()
        return loss

    # ------------------------------------------------------------------ HIP graph
    def _graph_body(self):
        """The launch sequence recorded into the step graph: STFT features of the mixed
        batch, forward, loss + its gradient, backward (everything between the mixing
        kernel and the all-reduce; no host synchronisation inside)."""
        self._stfts()
        self.forward()
        return self.loss_and_grad()

    def _ws_slot(self, l, bwd):
        """Layer l's hand-off workspace of the forward (bwd False) or BPTT pass.  (A method, not a
        lambda holding self: a reference cycle leaves a dropped trainer to the garbage collector,
        which could then free its device buffers in the middle of another trainer's graph capture.)"""
        return self.rnn_ws_all[int(bwd), l * self._w8:(l + 1) * self._w8]

    def capture(self):
        """Record STFT -> forward -> loss -> backward (~70 launches: persistent BiRNN
        kernels, gemm_gl GEMMs, attention, small kernels) as one HIP graph, replayed by
        step_graph().  The mixing kernel (its input pointer changes per batch), the RCCL
        all-reduce and Adam (its bias correction is a per-step host scalar) stay eager launches
        around the replay.  Bucketed data parallel: two graphs, split where the early bucket's
        all-reduce starts -- after the BPTT chain, which the side-stream dW_lin (forked and joined
        inside the first graph) runs beside; the second graph (the recurrent layers' weight-gradient
        launch) then runs beside that all-reduce.  Three buckets: a third graph -- the second graph holds
        the bias reduce and the upper layers' weight gradients, the third the lower layers' and the status
        flag, with the middle bucket's all-reduce started between them.  Call after at least one eager
        step(), so every workspace exists before the capture."""
        import gc

        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        g2 = torch.cuda.CUDAGraph() if self.buckets else None
        g3 = torch.cuda.CUDAGraph() if (self.buckets and self.dp_layer is not None) else None
        # no garbage collection while the stream is being captured: a collection that frees another
        # object's device memory mid-capture aborted the process (round 4, a dropped trainer's buffers)
        gc.collect()
        was_enabled = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.graph(g):
                self._graph_loss = self._graph_body()
                if g2 is None:
                    self.backward()
                else:
                    self.backward_early()
                    self._backward_fast("chain")
            if g2 is not None and g3 is None:
                with torch.cuda.graph(g2, pool=g.pool()):
                    self._backward_fast("wgrad")
                    self._status_flag()
            elif g3 is not None:
                with torch.cuda.graph(g2, pool=g.pool()):
                    self._backward_fast("upper")
                with torch.cuda.graph(g3, pool=g.pool()):
                    self._backward_fast("lower")
                    self._status_flag()
        finally:
            if was_enabled:
                gc.enable()
        torch.cuda.synchronize()
        self.graph, self.graph_late, self.graph_lower = g, g2, g3
        return g

    def step_graph(self, raw, gains, spk_idx):
        """step() with the captured graph: mixing, graph replay, all-reduce, Adam (bucketed: the
        early bucket's all-reduce between the first two replays, the middle one's between the second
        and the third)."""
        if getattr(self, "graph", None) is None:
            self.capture()
        self.spk.copy_(spk_idx)
        ops.mix_sources(raw, gains, out_src=self.src, out_mix=self.mix, stats_ws=self.stats)
        if self.fast and self._wb_stale():
            # parameters changed outside Adam since the capture
            self._weights_to_bf16()
        self.graph.replay()
        if self.graph_late is not None:
            self._early_bucket()
            self.graph_late.replay()
            if self.graph_lower is not None:
                self.allreduce_mid()
                self.graph_lower.replay()
            self.allreduce_late()
        else:
            self.allreduce()
        self.optimizer_step()
        return self._graph_loss

    def check(self):
        """Raise if a recurrence hand-off timed out, here or (data parallel) on a peer rank, since
        the last check: the guarded Adam already refused every update computed from then on.
        The refused steps are taken back out of step_count and the status word is reset, so the
        trainer can continue after the caller has handled it."""
        torch.cuda.synchronize()
        s, refused = (int(x) for x in self.status.tolist())
        if s or refused:
            self.status.zero_()
            self.rnn_ws_all.zero_()  # a timed-out launch's half-written hand-offs must not reach the next
            self.step_count -= refused
            where = "on this rank" if s else "on a data-parallel peer"
            raise RuntimeError(f"BiRNN hand-off timed out {where} (status {s}): {refused} update(s) refused")
