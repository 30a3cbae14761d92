"""Eval output path of the reference (Torch_multi/bss_test.py).

``reconstruct`` is the mask-apply + overlap-add iSTFT of ``bss_eval`` /
``bss_eval_cRM`` (EvalVer.py:36-75, cRM_EvalVer.py:69-106) in one kernel pass
(dl4ss_istft_apply); ``write_batch_output`` writes the reference's
``batch_output/`` wav naming (PCM16 via the stdlib ``wave`` module).

``cal`` scores a ``batch_output/`` directory with BSS-eval SDR (bss_test.py:12-61): the
reference's ``separation.bss_eval_sources`` is not vendored;
this build runs BSS_EVAL v3 on the GPU (``dl4ss_amd.bss``), parity unpinned against the
reference's copy and pinned against the restatement in ``oracle/bss_eval.py``.
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


def _read_wav(path):
    """PCM16 -> float64 in [-1, 1) (soundfile.read's default scaling, bss_test.py:30-36)."""
    with wave.open(path, "rb") as w:
        if w.getsampwidth() != 2:
            raise ValueError(f"{path}: only 16-bit PCM wavs are written by this build")
        return np.frombuffer(w.readframes(w.getnframes()), dtype="<i2").astype(np.float64) / 32768.0


def cal(path, aim_mix_number):
    """bss_test.py:12-61 (``add_slience_channel = 0``): per mixture index, the ``realTrue``
    wavs are the references and the ``pre`` wavs the estimates (sorted file order); one
    estimate against two references is repeated; returns the concatenated SDR arrays."""
    from dl4ss_amd import bss

    path = path if path.endswith(os.sep) else path + os.sep
    wavs = sorted(l for l in os.listdir(path) if l[-3:] == "wav")
    mix_number = len(set(l.split("_")[0] for l in wavs))
    print("num of mixed :", mix_number)
    sdr_sum = np.array([])
    for idx in range(mix_number):
        aim, pre = [], []
        for l in wavs:
            if l.split("_")[0] != str(idx):
                continue
            if "realTrue" in l:
                aim.append(_read_wav(path + l))
            if "pre" in l:
                pre.append(_read_wav(path + l))
        aim, pre = np.array(aim), np.array(pre)
        if pre.shape[0] == 1 and aim.shape[0] == 2:
            pre = pre.repeat(2, 0)
        sdr, sir, sar, perm = bss.bss_eval_sources(torch.from_numpy(aim).float(), torch.from_numpy(pre).float())
        result = (sdr[0], sir[0], sar[0], perm[0])
        print(result)
        sdr_sum = np.append(sdr_sum, result[0])
    print("SDR here:", sdr_sum.mean())
    return sdr_sum
