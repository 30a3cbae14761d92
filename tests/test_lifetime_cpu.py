"""Object lifetime invariant of the step objects: a dropped ``SepTrainer`` must be
freed by reference counting alone, with the garbage collector off.  A reference cycle (round 4: a
lambda holding ``self``) leaves the trainer to the collector, which may then run in the middle of
another trainer's ``torch.cuda.graph`` capture and free that trainer's buffers mid-capture (the
round-4 abort).  The trainers here are built on the CPU device: construction
only allocates buffers and asks the library host-only size queries (no GPU call)."""
import gc
import weakref

import pytest
import torch

from dl4ss_amd import engine, infer


@pytest.fixture
def no_gc():
    was = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


@pytest.mark.parametrize("cell,L,mode,precision", [("lstm", 4, "pit", "bf16"), ("lstm", 2, "label", "fp32"),
                                                   ("gru", 2, "label", "bf16s"), ("gru", 2, "crm", "bf16")])
def test_dropped_trainer_freed_by_refcount(no_gc, cell, L, mode, precision):
    net = engine.SepNet(cell=cell, num_layers=L, crm=mode == "crm", device="cpu")
    tr = engine.SepTrainer(net, 2, 2, 4000, mode=mode, precision=precision)
    # the host-side helpers the graph capture uses must not tie the trainer into a cycle either
    tr._ws_slot(0, False), tr._ws_slot(L - 1, True)
    ref = weakref.ref(tr)
    del tr
    assert ref() is None, [type(r).__name__ for r in gc.get_referrers(ref())]
    nref = weakref.ref(net)
    del net
    assert nref() is None


def test_dropped_recursive_extractor_freed_by_refcount(no_gc):
    net = engine.SepNet(cell="gru", num_layers=2, adjust=False, device="cpu")
    cnet = infer.ClassifierNet(129, 600, 3, 101, device="cpu")
    ex = infer.RecursiveExtractor(net, cnet, 1, 9, precision="mixed")
    refs = [weakref.ref(o) for o in (ex, ex.mask_net, ex.classifier, ex.mask_net.stack)]
    del ex
    assert all(r() is None for r in refs)


def test_recursive_extractor_modes():
    net = engine.SepNet(cell="gru", num_layers=2, adjust=False, device="cpu")
    cnet = infer.ClassifierNet(129, 600, 3, 101, device="cpu")
    ex = infer.RecursiveExtractor(net, cnet, 1, 9, precision="mixed")
    assert (ex.mask_net.precision, ex.mask_net.rnn_precision, ex.classifier.precision) == ("fp32", "bf16", "bf16")
    ex = infer.RecursiveExtractor(net, cnet, 1, 9, precision="bf16s")  # round 6: split-operand mask-net GEMMs
    assert (ex.mask_net.precision, ex.mask_net.rnn_precision, ex.classifier.precision) == ("bf16s", "bf16", "bf16")
    with pytest.raises(ValueError):
        infer.RecursiveExtractor(net, cnet, 1, 9, precision="bf16s2")


def test_step_plan_flags(monkeypatch):
    """The round-5 step-plan switches as the trainer derives them (host only): no gradient zeroing in
    the grouped bf16 backward, workspaces reused without a per-step fill from T >= 4, Adam-kept bf16
    weight copies, the two-term split of bf16s2 -- and each A/B override."""
    net = engine.SepNet(cell="lstm", num_layers=4, device="cpu")
    tr = engine.SepTrainer(net, 2, 2, 4000, mode="pit", precision="bf16")
    assert tr.zero_free and tr._gbeta == 0.0 and not tr._ws_fill and tr._shadow_on and not tr.split
    tr.params_changed()
    assert tr._wb_ver is None
    fp = engine.SepTrainer(net, 2, 2, 4000, mode="pit", precision="fp32")
    assert not fp.zero_free and fp._gbeta == 1.0 and not fp._shadow_on
    short = engine.SepTrainer(net, 2, 2, 300, mode="pit", precision="bf16")  # T = 3: a fill per step
    assert short.T < 4 and short._ws_fill
    deep = engine.SepTrainer(engine.SepNet(cell="lstm", num_layers=6, device="cpu"), 2, 2, 4000, precision="bf16")
    assert not deep.zero_free  # > 5 layers: per-layer weight-gradient GEMMs accumulate into the zeroed buffer
    gnet = engine.SepNet(cell="gru", num_layers=2, adjust=False, device="cpu")
    s2 = engine.SepTrainer(gnet, 2, 3, 4000, mode="pit", precision="bf16s2")
    assert s2.split and s2.split_x2 and s2.rnn_precision == "bf16" and s2.fast
    for name, attr in (("DL4SS_GRAD_ZERO", "zero_free"), ("DL4SS_ADAM_SHADOW", "_shadow_on")):
        monkeypatch.setenv(name, "1" if name == "DL4SS_GRAD_ZERO" else "0")
        assert not getattr(engine.SepTrainer(net, 2, 2, 4000, mode="pit", precision="bf16"), attr)
        monkeypatch.delenv(name)
    monkeypatch.setenv("DL4SS_WS_FILL", "1")
    assert engine.SepTrainer(net, 2, 2, 4000, mode="pit", precision="bf16")._ws_fill
