"""WSJ0-mix list reader + wav IO feeding the GPU mixing / STFT kernels.

Restates the real-data input of ``TDAA_beta/predata_fromList_cRM_123.py:90-255``:

* list files ``create-speaker-mixtures/mix_{k}_spk_{tr,cv,tt}.txt`` (``:98-105``), one mixture
  per line ``<path> <dB> <path> <dB> ...``; per line the speakers, gains and sample names
  come from the reference's three regexes (``:158-160``)::

      spk    = re.findall('/([0-9][0-9].)/', line)
      dB     = map(float, re.findall(' (.*?) ', line))
      sample = re.findall('/(.{8})\\.wav ', line)

  (the dB regex needs a space after the last value; a line ending in its last dB is read
  with one appended, which leaves lines that already end in a space unchanged);
* source wav = ``data_path/{train | eval_test}/<spk>/<sample>.wav`` (``:176-180``: 'test'
  reads eval_test, every other split train), first channel only (``:182-183``), cropped to
  MAX_LEN (``:187-188``);
* per source on the GPU (``dl4ss_mix_sources_rot``): mean removal and peak normalisation over
  the source's own length, on the train split with AUGMENT_DATA a rotation by a shift drawn
  ``random.sample(range(len), 1)[0]`` per source (``:197-200``), zero-padding to MAX_LEN, gain
  10^(dB/20), sum (``:192-237``);
  then the STFTs (mixture complex + magnitude, sources magnitude or complex) -- the batch
  the reference builds with librosa on the host (``:209-255``).

Resampling: the reference calls resampy ``kaiser_best`` when a wav is not at FRAME_RATE
(``:184-186``); resampy is absent here, so this build uses scipy's polyphase resampler
(``resample_poly``, Kaiser window beta 5) -- a documented divergence (parity unpinned for
non-8 kHz wavs; the WSJ0-2mix 8k lists are already at 8 kHz).
"""
import math
import os
import random
import re
import struct

import numpy as np
import torch

from . import ops

FRAME_RATE = 8000


def parse_line(line):
    """-> list of (speaker, sample_name, dB) in line order (predata_fromList_cRM_123.py:158-163)."""
    text = line.rstrip("\r\n")
    if not text.endswith(" "):
        text += " "
    spk = re.findall("/([0-9][0-9].)/", text)
    db = [float(x) for x in re.findall(" (.*?) ", text)]
    names = re.findall(r"/(.{8})\.wav ", text)
    if not (len(spk) == len(db) == len(names)) or not spk:
        raise ValueError(f"malformed mixture list line: {line!r}")
    return list(zip(spk, names, db))


def read_wav(path):
    """RIFF/WAVE reader -> (float64 signal of the first channel, rate).  PCM 8/16/24/32-bit
    (scaled like soundfile.read: int / 2^(bits-1); 8-bit is unsigned) and IEEE float 32/64."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{path}: not a RIFF/WAVE file")
    pos, fmt, payload = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack("<I", data[pos + 4:pos + 8])[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = struct.unpack("<HHIIHH", body[:16])
        elif cid == b"data":
            payload = body
        pos += 8 + size + (size & 1)
    if fmt is None or payload is None:
        raise ValueError(f"{path}: missing fmt or data chunk")
    tag, nch, rate, _, _, bits = fmt
    if tag == 0xFFFE:  # WAVE_FORMAT_EXTENSIBLE: the sub-format's first two bytes are the tag
        tag = 3 if bits in (32, 64) and b"\x03\x00" in data[:200] else 1
    if tag == 3:
        x = np.frombuffer(payload, dtype="<f4" if bits == 32 else "<f8").astype(np.float64)
    elif tag == 1:
        if bits == 8:
            x = (np.frombuffer(payload, dtype=np.uint8).astype(np.float64) - 128.0) / 128.0
        elif bits == 16:
            x = np.frombuffer(payload, dtype="<i2").astype(np.float64) / 32768.0
        elif bits == 24:
            b = np.frombuffer(payload, dtype=np.uint8).reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            x = np.where(v >= 1 << 23, v - (1 << 24), v).astype(np.float64) / float(1 << 23)
        elif bits == 32:
            x = np.frombuffer(payload, dtype="<i4").astype(np.float64) / float(1 << 31)
        else:
            raise ValueError(f"{path}: {bits}-bit PCM unsupported")
    else:
        raise ValueError(f"{path}: wave format tag {tag} unsupported")
    n = len(x) // nch
    return x[:n * nch].reshape(n, nch)[:, 0].copy(), rate


def write_wav(path, x, rate=FRAME_RATE):
    """16-bit PCM mono writer (clipped to [-1, 1))."""
    q = np.clip(np.round(np.asarray(x, dtype=np.float64) * 32768.0), -32768, 32767).astype("<i2")
    hdr = struct.pack("<4sI4s4sIHHIIHH4sI", b"RIFF", 36 + 2 * len(q), b"WAVE", b"fmt ", 16, 1, 1, rate, 2 * rate, 2,
                      16, b"data", 2 * len(q))
    with open(path, "wb") as f:
        f.write(hdr + q.tobytes())


def resample(x, rate, target=FRAME_RATE):
    if rate == target:
        return x
    from scipy.signal import resample_poly
    g = math.gcd(int(rate), int(target))
    return resample_poly(x, target // g, int(rate) // g)


def source_path(data_path, split, spk, name):
    sub = "eval_test" if split == "test" else "train"
    return os.path.join(data_path, sub, spk, name + ".wav")


class ListBatches:
    """Batches of one list file (one mixture size k): host arrays ready for the GPU step.

    Each batch: raw (B, k, max_len) float32 (cropped, zero-padded, NOT yet normalised),
    lengths (B, k) int32, gains (B, k) float32 = 10^(dB/20), speakers / sample names per
    row.  ``batch_total = len(lines) // B`` batches per epoch (the reference's
    ``batch_mix``); ``shuffle`` reorders the lines once per epoch (config.SHUFFLE_BATCH).
    augment: draw each source's rotation (shifts (B, k) int32 in the batch, else None)."""

    def __init__(self, list_path, data_path, split, batch, max_len, shuffle=False, seed=1, augment=False):
        with open(list_path) as f:
            self.lines = [l for l in f.readlines() if l.strip()]
        self.items = [parse_line(l) for l in self.lines]
        ks = {len(it) for it in self.items}
        if len(ks) != 1:
            raise ValueError("a list file holds mixtures of one size (mix_{k}_spk_*.txt)")
        self.k = ks.pop()
        self.data_path, self.split, self.B, self.max_len = data_path, split, batch, max_len
        self.shuffle, self.rng = shuffle, random.Random(seed)
        self.augment = augment
        self.batch_total = len(self.items) // batch

    def load(self, item):
        raw = np.zeros((self.k, self.max_len), dtype=np.float32)
        lens = np.zeros(self.k, dtype=np.int32)
        shifts = np.zeros(self.k, dtype=np.int32)
        for j, (spk, name, _) in enumerate(item):
            x, rate = read_wav(source_path(self.data_path, self.split, spk, name))
            x = resample(x, rate)[:self.max_len]
            raw[j, :len(x)] = x
            lens[j] = len(x)
            if self.augment:  # predata_fromList_cRM_123.py:198-199, drawn per source in line order
                shifts[j] = random.sample(range(len(x)), 1)[0]
        gains = np.array([10.0 ** (db / 20.0) for _, _, db in item], dtype=np.float32)
        return raw, lens, gains, shifts

    def __iter__(self):
        order = list(range(len(self.items)))
        if self.shuffle:
            self.rng.shuffle(order)
        for bi in range(self.batch_total):
            rows = [self.items[i] for i in order[bi * self.B:(bi + 1) * self.B]]
            loaded = [self.load(it) for it in rows]
            yield dict(raw=np.stack([l[0] for l in loaded]), lengths=np.stack([l[1] for l in loaded]),
                       gains=np.stack([l[2] for l in loaded]), speakers=[[s for s, _, _ in it] for it in rows],
                       names=[[n for _, n, _ in it] for it in rows],
                       shifts=np.stack([l[3] for l in loaded]) if self.augment else None)


def features(batch, device, complex_sources=False):
    """One list batch -> device tensors: normalised sources (B,k,N), mixture (B,N), mixture
    STFT complex (B,T,F,2) + magnitude (B,T,F), source magnitude (B,k,T,F) (or complex
    (B,k,T,F,2) for the cRM targets)."""
    raw = torch.from_numpy(batch["raw"]).to(device)
    gains = torch.from_numpy(batch["gains"]).to(device)
    lens = torch.from_numpy(batch["lengths"]).to(device)
    shifts = batch.get("shifts")
    shifts = None if shifts is None else torch.from_numpy(np.ascontiguousarray(shifts, np.int32)).to(device)
    B, K, N = raw.shape
    src, mix = ops.mix_sources(raw, gains, lengths=lens, shifts=shifts)
    Xc, Xm = ops.stft(mix, complex_out=True, mag_out=True)
    if complex_sources:
        Sc, _ = ops.stft(src.view(B * K, N), complex_out=True, mag_out=False)
        S = Sc.view(B, K, *Sc.shape[1:])
    else:
        _, Sm = ops.stft(src.view(B * K, N), complex_out=False, mag_out=True)
        S = Sm.view(B, K, *Sm.shape[1:])
    return dict(src=src, mix=mix, mix_complex=Xc, mix_mag=Xm, src_spec=S)
