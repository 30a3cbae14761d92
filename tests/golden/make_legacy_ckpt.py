"""Hand-built torch-0.3 / Python-2 checkpoint fixtures (``python tests/golden/make_legacy_ckpt.py``).

The reference saves one ``state_dict`` per module with ``torch.save`` under Python 2 and
torch 0.3 (``TDAA_beta/main_run_sstune_EvalVer.py:677-690``; loaded back at ``:545-554``
with ``map_location={'cuda:1': 'cuda:0'}``).  No such file ships with the reference and
neither interpreter exists here, so this script writes the bytes that combination produces,
opcode by opcode (the legacy, pre-zip serialization):

  1. pickle(MAGIC_NUMBER)      protocol 2, a py2 ``long`` -> LONG1
  2. pickle(1001)              PROTOCOL_VERSION
  3. pickle(sys_info)          {'protocol_version', 'little_endian', 'type_sizes'} (py2 ``str``
                               keys -> SHORT_BINSTRING)
  4. pickle(state_dict)        ``collections.OrderedDict`` reduced from a list of [key, value]
                               pairs (py2 OrderedDict.__reduce__); every tensor is
                               ``torch._utils._rebuild_tensor(storage, offset, size, stride)``
                               (0.3's 4-argument form, before _rebuild_tensor_v2) and every
                               storage a persistent id ('storage', torch.cuda.FloatStorage,
                               key, 'cuda:1', numel, None); globals memoised (BINPUT / BINGET)
  5. pickle(sorted storage keys)
  6. per storage: int64 element count + raw little-endian float32 data

The tensors are a BiGRU-2L mask net at H = 8, E = 4 (F = 129: small enough to commit) with
the reference's key names; the values are seeded numpy draws, also saved as
``expected.npz`` for the loader test (tests/test_checkpoint_cpu.py).
"""
import io
import os
import struct
import sys
from collections import OrderedDict

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "legacy_py2_torch03")
MAGIC_NUMBER = 0x1950A86A20F9469CFC6C


class P2:
    """Minimal protocol-2 opcode writer with py2-style memoisation."""

    def __init__(self):
        self.b = io.BytesIO()
        self.memo = {}

    def op(self, x):
        self.b.write(x)

    def put(self):
        n = len(self.memo)
        self.memo[("#", n)] = n
        self.op(b"q" + bytes([n]) if n < 256 else b"r" + struct.pack("<I", n))
        return n

    def proto(self):
        self.op(b"\x80\x02")

    def stop(self):
        self.op(b".")

    def glob(self, module, name):
        key = ("g", module, name)
        if key in self.memo:
            n = self.memo[key]
            self.op(b"h" + bytes([n]) if n < 256 else b"j" + struct.pack("<I", n))
            return
        self.op(b"c" + module.encode() + b"\n" + name.encode() + b"\n")
        self.memo[key] = self.put()

    def string(self, s):  # py2 str
        d = s.encode()
        assert len(d) < 256
        self.op(b"U" + bytes([len(d)]) + d)
        self.put()

    def int(self, v):
        if 0 <= v < 256:
            self.op(b"K" + bytes([v]))
        elif 0 <= v < 65536:
            self.op(b"M" + struct.pack("<H", v))
        elif -2 ** 31 <= v < 2 ** 31:
            self.op(b"J" + struct.pack("<i", v))
        else:  # py2 long
            n = (v.bit_length() + 8) // 8
            self.op(b"\x8a" + bytes([n]) + v.to_bytes(n, "little", signed=True))

    def tuple_(self, items):
        if len(items) == 0:
            self.op(b")")
            return
        if len(items) <= 3:
            for it in items:
                it()
            self.op({1: b"\x85", 2: b"\x86", 3: b"\x87"}[len(items)])
        else:
            self.op(b"(")
            for it in items:
                it()
            self.op(b"t")
        self.put()


def dump_scalar(w, fn):
    w.proto()
    fn()
    w.stop()


def write_state_dict(path, sd):
    keys = {}  # storage key (py2: str(obj._cdata)) per tensor
    base = 94_210_000_000_000
    for i, k in enumerate(sd):
        keys[k] = str(base + 48 * i)
    w = P2()
    # 1-3: magic, protocol version, sys_info
    dump_scalar(w, lambda: w.int(MAGIC_NUMBER))
    w.memo.clear()
    dump_scalar(w, lambda: w.int(1001))
    w.memo.clear()
    w.proto()
    w.op(b"}")
    w.put()
    w.op(b"(")
    w.string("protocol_version")
    w.int(1001)
    w.string("little_endian")
    w.op(b"\x88")
    w.string("type_sizes")
    w.op(b"}")
    w.put()
    w.op(b"(")
    for name, size in (("short", 2), ("int", 4), ("long", 8)):
        w.string(name)
        w.int(size)
    w.op(b"u")
    w.op(b"u")
    w.stop()
    w.memo.clear()
    # 4: the OrderedDict
    w.proto()
    w.glob("collections", "OrderedDict")
    w.op(b"]")  # the (items,) list of [key, value] pairs
    w.put()
    w.op(b"(")
    for k, a in sd.items():
        w.op(b"]")
        w.put()
        w.op(b"(")
        w.string(k)
        # _rebuild_tensor(storage, storage_offset, size, stride)
        w.glob("torch._utils", "_rebuild_tensor")
        w.op(b"(")
        # persistent id of the storage
        w.op(b"(")
        w.string("storage")
        w.glob("torch.cuda", "FloatStorage")
        w.string(keys[k])
        w.string("cuda:1")
        w.int(int(a.size))
        w.op(b"N")
        w.op(b"t")
        w.put()
        w.op(b"Q")  # BINPERSID
        w.int(0)
        w.tuple_([(lambda v=v: w.int(v)) for v in a.shape])
        strides = [int(np.prod(a.shape[i + 1:])) for i in range(a.ndim)]
        w.tuple_([(lambda v=v: w.int(v)) for v in strides])
        w.op(b"t")
        w.put()
        w.op(b"R")
        w.put()
        w.op(b"e")  # APPENDS: [key, tensor]
    w.op(b"e")
    w.op(b"\x85")  # (items,)
    w.put()
    w.op(b"R")
    w.put()
    w.stop()
    w.memo.clear()
    # 5: storage keys, sorted
    w.proto()
    w.op(b"]")
    w.put()
    w.op(b"(")
    for key in sorted(keys.values()):
        w.string(key)
    w.op(b"e")
    w.stop()
    # 6: raw storages in key order
    by_key = {keys[k]: a for k, a in sd.items()}
    for key in sorted(by_key):
        a = np.ascontiguousarray(by_key[key], dtype="<f4")
        w.op(struct.pack("<q", a.size))
        w.op(a.tobytes())
    with open(path, "wb") as f:
        f.write(w.b.getvalue())


def module_dicts(H=8, E=4, F=129, layers=2, num_labels=101, seed=3):
    r = np.random.Generator(np.random.PCG64(seed))
    mix = OrderedDict()
    for l in range(layers):
        D = F if l == 0 else 2 * H
        for sfx in ("", "_reverse"):
            for kind, shape in (("weight_ih", (3 * H, D)), ("weight_hh", (3 * H, H)), ("bias_ih", (3 * H,)),
                                ("bias_hh", (3 * H,))):
                mix[f"layer.{kind}_l{l}{sfx}"] = r.uniform(-0.3, 0.3, size=shape).astype(np.float32)
    mix["Linear.weight"] = r.uniform(-0.2, 0.2, size=(F * E, 2 * H)).astype(np.float32)
    mix["Linear.bias"] = r.uniform(-0.2, 0.2, size=(F * E,)).astype(np.float32)
    emb = OrderedDict(**{"layer.weight": r.standard_normal((num_labels, E)).astype(np.float32)})
    adj = OrderedDict(**{"layer.weight": r.uniform(-0.2, 0.2, size=(E, 2 * H + E)).astype(np.float32)})
    return mix, emb, adj


def main():
    os.makedirs(OUT, exist_ok=True)
    mix, emb, adj = module_dicts()
    # file names of cRM_EvalVer.py:615-618 / selfSS_dB.py:432-434
    write_state_dict(os.path.join(OUT, "param_mix101_WSJ0_hidden3d_180"), mix)
    write_state_dict(os.path.join(OUT, "param_mix101_WSJ0_emblayer_180"), emb)
    write_state_dict(os.path.join(OUT, "param_mix101_WSJ0_adjlayer_180"), adj)
    flat = {f"mix.{k}": v for k, v in mix.items()}
    flat.update({f"emb.{k}": v for k, v in emb.items()})
    flat.update({f"adj.{k}": v for k, v in adj.items()})
    np.savez_compressed(os.path.join(OUT, "expected.npz"), **flat)
    print("wrote", OUT, file=sys.stderr)


if __name__ == "__main__":
    main()
