"""The dl4ss::* torch.library custom ops (dl4ss_amd/library.py): every op is
registered with a schema, shapes propagate through the fake (meta) kernels without a GPU, and a
CPU tensor is refused (there is no CPU implementation: the product path fails loudly)."""
import pytest
import torch

from dl4ss_amd import library as L


def test_every_op_registered_with_schema():
    for name in L.OPS:
        op = getattr(torch.ops.dl4ss, name).default
        assert op._schema.name == f"dl4ss::{name}"


def test_meta_shapes():
    m = dict(device="meta")
    x = torch.empty(3, 32000, **m)
    assert torch.ops.dl4ss.stft_mag(x, True).shape == (3, 251, 129)
    assert torch.ops.dl4ss.stft_complex(x, False).shape == (3, 251, 129, 2)
    S = torch.empty(3, 251, 129, 2, **m)
    assert torch.ops.dl4ss.istft(S, False).shape == (3, 32000)
    aux = torch.empty(6, 251, 129, **m)
    assert torch.ops.dl4ss.istft_apply(S, aux, 2, False, False).shape == (6, 32000)
    src, mix = torch.ops.dl4ss.mix_sources(torch.empty(3, 2, 32000, **m), torch.empty(3, 2, **m))
    assert src.shape == (3, 2, 32000) and mix.shape == (3, 32000)
    xb = torch.empty(2, 17, 129, **m)
    for cell, g in (("lstm", 4), ("gru", 3)):
        out, hprev, act, cs = torch.ops.dl4ss.birnn_layer(
            xb, torch.empty(2 * g * 300, 129, **m), torch.empty(2 * g * 300, **m), torch.empty(2 * g * 300, 300, **m),
            torch.empty(2 * g * 300, **m), cell, 300, "bf16")
        assert out.shape == (2, 17, 600) and act.shape == (2, 17, 2, 1200)
        assert cs.shape == ((2, 17, 2, 300) if cell == "lstm" else (0,))
    v = torch.ops.dl4ss.linear_tanh(torch.empty(34, 600, **m), torch.empty(6450, 600, **m), torch.empty(6450, **m),
                                    "fp32")
    assert v.shape == (34, 6450)
    V = torch.empty(4, 129 * 17, 50, **m)
    assert torch.ops.dl4ss.attention_dot(V, torch.empty(4, 50, **m), False).shape == (4, 129 * 17)
    assert torch.ops.dl4ss.attention_dot(V, torch.empty(4, 100, **m), True).shape == (4, 129 * 17, 2)
    mask, idx, cnt = torch.ops.dl4ss.top_k_mask(torch.empty(5, 101, **m), 0.5, 3)
    assert mask.shape == (5, 101) and idx.shape == (5, 3) and idx.dtype == torch.int32 and cnt.shape == (5,)


def test_cpu_tensor_is_refused():
    with pytest.raises((NotImplementedError, RuntimeError)):
        torch.ops.dl4ss.stft_mag(torch.zeros(1, 4000), False)
