"""WSJ0-mix list reader + wav IO (TDAA_beta/predata_fromList_cRM_123.py:90-255):
line parsing with the reference's regexes, wav round trips, batch assembly (host side)."""
import os
import struct

import numpy as np
import pytest

from dl4ss_amd import wsj0list as wl


def _dataset(tmp_path, rate=8000):
    rng = np.random.default_rng(0)
    data = tmp_path / "data"
    lines = []
    lens = {"01aa0101": 9000, "02bb0202": 12000, "03cc0303": 5000, "04dd0404": 12000}
    spk = {"01aa0101": "01a", "02bb0202": "02b", "03cc0303": "03c", "04dd0404": "04d"}
    for name, n in lens.items():
        d = data / "train" / spk[name]
        d.mkdir(parents=True, exist_ok=True)
        wl.write_wav(str(d / f"{name}.wav"), 0.3 * rng.standard_normal(n * rate // 8000).clip(-3, 3) / 3, rate)
    lines.append("wsj0/si_tr_s/01a/01aa0101.wav 1.5 wsj0/si_tr_s/02b/02bb0202.wav -1.5\n")
    lines.append("wsj0/si_tr_s/03c/03cc0303.wav 0.25 wsj0/si_tr_s/04d/04dd0404.wav -0.25 \n")
    lines.append("wsj0/si_tr_s/02b/02bb0202.wav 2 wsj0/si_tr_s/03c/03cc0303.wav -2\n")
    lst = tmp_path / "mix_2_spk_tr.txt"
    lst.write_text("".join(lines))
    return str(lst), str(data), lens


def test_parse_line_reference_regexes():
    it = wl.parse_line("wsj0/si_tr_s/01t/01to030v.wav 0.26456 wsj0/si_tr_s/011/011o0319.wav -0.26456\n")
    assert it == [("01t", "01to030v", 0.26456), ("011", "011o0319", -0.26456)]
    assert wl.parse_line("a/40a/40aa0101.wav 1 b/41b/41bb0101.wav 2 c/42c/42cc0101.wav 3 \n")[2] == ("42c", "42cc0101",
                                                                                                   3.0)
    with pytest.raises(ValueError):
        wl.parse_line("garbage line\n")


def test_wav_round_trip_and_formats(tmp_path):
    x = np.linspace(-0.9, 0.9, 1001)
    p = str(tmp_path / "a.wav")
    wl.write_wav(p, x, 8000)
    y, rate = wl.read_wav(p)
    assert rate == 8000 and np.abs(y - x).max() <= 1 / 32768
    # 2-channel float32 -> first channel
    st = np.stack([x, -x], 1).astype("<f4")
    hdr = struct.pack("<4sI4s4sIHHIIHH4sI", b"RIFF", 36 + st.nbytes, b"WAVE", b"fmt ", 16, 3, 2, 16000, 16000 * 8, 8,
                      32, b"data", st.nbytes)
    q = str(tmp_path / "f.wav")
    with open(q, "wb") as f:
        f.write(hdr + st.tobytes())
    y, rate = wl.read_wav(q)
    assert rate == 16000 and np.abs(y - x.astype(np.float32)).max() == 0
    assert len(wl.resample(y, rate)) == 501


def test_list_batches(tmp_path):
    lst, data, lens = _dataset(tmp_path)
    lb = wl.ListBatches(lst, data, "train", batch=2, max_len=10000)
    assert lb.k == 2 and lb.batch_total == 1
    (b,) = list(lb)
    assert b["raw"].shape == (2, 2, 10000) and b["raw"].dtype == np.float32
    assert b["lengths"].tolist() == [[9000, 10000], [5000, 10000]]
    assert np.allclose(b["gains"], [[10 ** (1.5 / 20), 10 ** (-1.5 / 20)], [10 ** (0.25 / 20), 10 ** (-0.25 / 20)]])
    assert b["speakers"] == [["01a", "02b"], ["03c", "04d"]]
    x, _ = wl.read_wav(os.path.join(data, "train", "01a", "01aa0101.wav"))
    assert np.array_equal(b["raw"][0, 0, :9000], x.astype(np.float32)) and not b["raw"][0, 0, 9000:].any()
