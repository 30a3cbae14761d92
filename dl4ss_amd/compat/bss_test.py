"""Eval output path of the reference (Torch_multi/bss_test.py).

``reconstruct`` is the mask-apply + overlap-add iSTFT of ``bss_eval`` /
``bss_eval_cRM`` (EvalVer.py:36-75, cRM_EvalVer.py:69-106) in one kernel pass
(dl4ss_istft_apply); ``write_batch_output`` writes the reference's
``batch_output/`` wav naming (PCM16 via the stdlib ``wave`` module).

``cal`` needs BSS-eval SDR (``separation.bss_eval_sources``), a dependency the
reference does not vendor: parity unpinned, listed as the
next row; it raises until that row is built.
"""
import os
import wave

import numpy as np
import torch

from dl4ss_amd import _lib


def reconstruct(pred, mix_complex, crm=False, conj=False):
    """pred (B, K, T, F) masked magnitude -- or (B, K, T, F, 2) complex mask when crm --
    and the mixture spectrum (B, T, F, 2) [re, im] -> waveforms (B, K, 128 (T-1))."""
    pred = pred.float().contiguous()
    X = mix_complex.float().contiguous()
    B, K, T = pred.shape[:3]
    y = torch.empty(B, K, 128 * (T - 1), device=pred.device)
    _lib.call("dl4ss_istft_apply", _lib.ptr(X), _lib.ptr(pred), B * K, K, T, 1 if crm else 0, int(conj),
              _lib.ptr(y), _lib.stream_ptr())
    return y


def _write_wav(path, x, rate=8000):
    x = np.clip(np.asarray(x, dtype=np.float64), -1.0, 1.0)
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(rate)
        w.writeframes((x * 32767.0).astype("<i2").tobytes())


def write_batch_output(path, waves_pred, names, mix_wav=None, clean=None, rate=8000):
    """``{idx}_{spk}_pre.wav`` per estimate, ``{idx}_{spk}_realTrue.wav`` per clean
    source, ``{idx}_True_mix.wav`` (EvalVer.py:44-72 naming)."""
    os.makedirs(path, exist_ok=True)
    w = waves_pred.cpu().numpy() if torch.is_tensor(waves_pred) else np.asarray(waves_pred)
    for b, row in enumerate(names):
        for k, spk in enumerate(row):
            _write_wav(os.path.join(path, f"{b}_{spk}_pre.wav"), w[b, k], rate)
            if clean is not None:
                _write_wav(os.path.join(path, f"{b}_{spk}_realTrue.wav"), clean[b][spk], rate)
        if mix_wav is not None:
            _write_wav(os.path.join(path, f"{b}_True_mix.wav"), mix_wav[b], rate)


def cal(path, aim_mix_number):
    raise NotImplementedError("bss_test.cal needs BSS-eval SDR (separation.bss_eval_sources, not vendored by the "
                              "reference): SURVEY section 8f row f2, not built yet")
