"""LDS bank-conflict model of the packed recurrence kernels' per-step LDS accesses (birnn.hip,
rnn_fwd_pk_kernel / rnn_bwd_pk_kernel) at the C2 plan (BiLSTM, B = 32, H = 300: BC = 4, J = 20,
NG = 15) and the BiGRU plan, from the lane groups and bank functions of
MI355X_MICROARCH.md section LDS (the table of lane groups per instruction).

For every access of a step: LDS-array cycles, the conflict-free minimum, and the extra
(conflict) cycles -- the quantity SQ_LDS_BANK_CONFLICT counts.  Layouts are given by the
same index formulas as the kernel, with the padding / swizzle knobs the kernel uses, so a
layout change can be checked here before it goes to the GPU.

  python tools/lds_banks.py [--old]      # --old: the round-2 layouts (default: the shipped ones)
"""
import argparse

# lane groups (each one LDS cycle when conflict-free) and bank count per instruction
G32 = [list(range(0, 32)), list(range(32, 64))]
B128_READ = [[0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)),
             list(range(4, 12)) + [16, 17, 18, 19] + list(range(28, 32)),
             [32, 33, 34, 35, 44, 45, 46, 47] + list(range(52, 60)),
             list(range(36, 44)) + [48, 49, 50, 51] + list(range(60, 64))]
INSTR = {
    "ds_read_b32": (G32, 32, 1),
    "ds_read_b64": (G32, 64, 2),
    "ds_read_b128": (B128_READ, 64, 4),
    "ds_write_b32": ([list(range(i, i + 32)) for i in (0, 32)], 32, 1),
    "ds_write_b64": ([list(range(i, i + 16)) for i in range(0, 64, 16)], 32, 2),
    "ds_write_b128": ([list(range(i, i + 8)) for i in range(0, 64, 8)], 32, 4),
    "ds_write_b16": ([list(range(i, i + 32)) for i in (0, 32)], 32, 1),
}


def cycles(instr, addr):
    """addr: per lane byte address or None (inactive).  Returns (cycles, min_cycles)."""
    groups, nb, nd = INSTR[instr]
    cyc = mn = 0
    for g in groups:
        banks = {}
        act = False
        for l in g:
            a = addr[l]
            if a is None:
                continue
            act = True
            for i in range(nd):
                dw = a // 4 + i
                banks.setdefault(dw % nb, set()).add(dw)
        if act:
            cyc += max(len(v) for v in banks.values())
            mn += 1
    return cyc, mn


def wave_lanes(w):
    return [w * 64 + l for l in range(64)]


def fwd_accesses(cell, old, XW=False, BC=4, J=20, NG=15, H=300):
    ngate = 4 if cell == "lstm" else 3
    R = ngate * J
    MT = (R + 15) // 16
    KSMAX = 10
    SHB = KSMAX * 32 + 8 if old else KSMAX * 32 + 8  # bf16 row stride of the h B image
    shb = 0
    sgate = 2 * 8 * SHB  # bytes (smem float offset 8*SHB)
    sgs = MT * 16 if old else MT * 16 + 4  # sgate row stride (floats)
    sin = sgate + 4 * BC * sgs
    acc = []
    NPW = 2
    # F1 gather tail: polling waves 4 and 7, GLK = 2 sweeps, three 4-B stores per lane
    GLK = (BC + NPW - 1) // NPW
    n16 = BC * NG * 4
    for pwv in range(NPW):
        for g in range(GLK):
            for part in range(3):
                addr = []
                for lane in range(64):
                    idx = lane + 64 * (g * NPW + pwv)
                    if idx >= n16:
                        addr.append(None)
                        continue
                    b, pw, pp = idx // (NG * 4), (idx // 4) % NG, idx % 4
                    k0 = pw * J + 6 * pp
                    nv = max(0, min(min(6, J - 6 * pp), H - k0))
                    addr.append(shb + 2 * (b * SHB + k0) + 4 * part if nv > 2 * part else None)
                acc.append((f"F1 gather-tail store {part} (wave {4 if pwv == 0 else 7}, sweep {g})", "ds_write_b32",
                            addr, 1))
    # F2 matvec B reads, MT waves
    for ks in range(KSMAX):
        # new: B-image rows >= BC (all zero) are read from row BC (one shared zero row: broadcast)
        addr = [shb + 2 * ((l & 15 if old else min(l & 15, BC)) * SHB + 8 * (l >> 4) + ks * 32) for l in range(64)]
        acc.append((f"F2 matvec B read ks={ks}", "ds_read_b128", addr, MT))
    # F3 sgate stores (col < BC lanes)
    for tile in range(MT):
        addr = [sgate + 4 * ((l & 15) * sgs + tile * 16 + (l >> 4) * 4) if (l & 15) < BC else None for l in range(64)]
        acc.append((f"F3 sgate store tile {tile}", "ds_write_b128", addr, 1))
    # F4 cell phase: sin float4 (waves 0-1), sgate scalar reads
    for w in range(BC * 32 // 64):
        if old:
            addr = [sin + 16 * (w * 64 + l) for l in range(64)]
        else:  # round 4: dense records, cell = b * J + u
            addr = [sin + 16 * (((w * 64 + l) >> 5) * J + (l & 31)) if (l & 31) < J else None for l in range(64)]
        acc.append((f"F4 sin read wave {w}", "ds_read_b128", addr, 1))
        for q in range(ngate):
            addr = []
            for l in range(64):
                tid = w * 64 + l
                cb, cu = tid >> 5, tid & 31
                addr.append(sgate + 4 * (cb * sgs + q * J + cu) if cu < J else None)
            acc.append((f"F4 sgate read q={q} wave {w}", "ds_read_b32", addr, 1))
    # F6 prefetch commit into sin (non-XW): item q of prefetch waves 5-6
    if not XW:
        NPF = 128
        NQ = (BC * 20 * 4 + NPF - 1) // NPF
        for wv in (5, 6):
            for q in range(NQ):
                addr = []
                for lane in range(64):
                    i = (wv - 5) * 64 + lane + q * NPF
                    if old:
                        gate, c = i // (BC * J), i % (BC * J)
                    else:  # new: the four gates of a cell on consecutive lanes
                        gate, c = i & 3, i >> 2
                    if gate >= ngate or c >= BC * J:
                        addr.append(None)
                        continue
                    dst = ((c // J) * 32 + c % J) * 4 + gate if old else c * 4 + gate
                    addr.append(sin + 4 * dst)
                acc.append((f"F6 prefetch commit wave {wv} q={q}", "ds_write_b32", addr, 1))
    return acc


def xw_accesses(old, BC=4, XK=20, J=20, R=80, xfinal_layout="r4"):
    SXB = 640 if old else 656  # bf16 row stride of the DMA'd input rows (new: 82 16-B chunks)
    NXQ = (BC * (SXB // 8) + 127) // 128
    sxb = 0
    # the zero row after the ring, new: at the bank offset row BC would have
    sxz = 2 * (4 * NXQ * 128 * 8 + (0 if old else (BC * SXB) % 128))
    acc = []
    for ks in range(XK):
        addr = []
        for l in range(64):
            row = l & 15
            base = (sxb + 2 * row * SXB) if row < BC else sxz
            addr.append(base + 2 * (8 * (l >> 4) + ks * 32))
        acc.append((f"XW B read ks={ks}", "ds_read_b128", addr, 5))
    # xfinal: the block epilogue writes G of SPB = 16 / BC steps once per block (x 1 / SPB per step):
    # lane (o = n / BC, b = n % BC, h = lane >> 4) stores element e of rows t * 16 + 4 h + e into step
    # slot o.  "r3": [b * 32 + u][4] records in 512-float slabs (16 lanes on one bank); "r4": dense
    # records (cell = b * J + u), slab stride BC * 128 + 4
    spb = 16 // BC
    for t in range((R + 15) // 16):
        for e in range(4):
            addr = []
            for l in range(64):
                n, h = l & 15, l >> 4
                o, b, rr = n // BC, n % BC, t * 16 + 4 * h + e
                if rr >= R:
                    addr.append(None)
                elif xfinal_layout == "r3":
                    addr.append(4 * (o * BC * 128 + (b * 32 + rr % J) * 4 + rr // J))
                else:
                    addr.append(4 * (o * (BC * 128 + 4) + (b * J + rr % J) * 4 + rr // J))
            acc.append((f"XW xfinal store tile {t} e={e} (per block)", "ds_write_b32", addr, 1 / spb))
    return acc


def bwd_accesses(cell, old, BC=4, J=20, NG=15, H=300):
    ngate = 4 if cell == "lstm" else 3
    KSRMAX = 3
    SDG = KSRMAX * 32 + 8  # bf16
    WSPAN = 80
    wsp = WSPAN if old else WSPAN + 4
    BSL_N = 6  # round 4: slot partials summed by the polling lanes (BSL_Q = 5 BC lanes per slot)
    sdgb = 0
    sdh = 2 * 8 * SDG
    wsc = sdh + 4 * ((16 * BC * J + 3) & ~3)
    sop = wsc + 4 * 4 * BC * wsp
    acc = []
    # B2 operand record reads (cell lanes, waves 0-1)
    for w in range(BC * 32 // 64):
        for half in range(2):
            if old:
                addr = [sop + 4 * ((w * 64 + l) * 8 + 4 * half) for l in range(64)]
            else:  # round 4: dense cell index b * J + u
                addr = []
                for l in range(64):
                    cb, cu = (w * 64 + l) >> 5, l & 31
                    addr.append(sop + 4 * (half * (BC * 32 * 4 + 16) + (cb * J + cu) * 4) if cu < J else None)
            acc.append((f"B2 operand read {half} wave {w}", "ds_read_b128", addr, 1))
        for i in range(16 if old else BSL_N):
            addr = []
            for l in range(64):
                tid = w * 64 + l
                cb, cu = tid >> 5, tid & 31
                addr.append(sdh + 4 * (i * BC * J + cb * J + cu) if cu < J else None)
            acc.append((f"B3 partial read {i} wave {w}", "ds_read_b32", addr, 1))
        for q in range(ngate):
            addr = []
            for l in range(64):
                tid = w * 64 + l
                cb, cu = tid >> 5, tid & 31
                addr.append(sdgb + 2 * (cb * SDG + q * J + cu) if cu < J else None)
            acc.append((f"B4 dgh store q={q} wave {w}", "ds_write_b16", addr, 1))
    # B5 MFMA B reads, 4 waves
    for ks in range(KSRMAX):
        addr = [sdgb + 2 * ((l & 15 if old else min(l & 15, BC)) * SDG + 8 * (l >> 4) + ks * 32) for l in range(64)]
        acc.append((f"B5 MFMA B read ks={ks}", "ds_read_b128", addr, 4))
    # B6 accumulator stores into the wave-private transpose (col < BC lanes), 5 tiles
    for t2 in range(5):
        addr = [wsc + 4 * ((l & 15) * wsp + t2 * 16 + 4 * (l >> 4)) if (l & 15) < BC else None for l in range(64)]
        acc.append((f"B6 transpose store t2={t2}", "ds_write_b128", addr, 4))
    # B7 transpose reads
    NQW = BC * WSPAN // 4
    for e0 in range(0, NQW, 64):
        addr = []
        for l in range(64):
            e = e0 + l
            if e >= NQW:
                addr.append(None)
                continue
            bb, k = e // (WSPAN // 4), 4 * (e % (WSPAN // 4))
            addr.append(wsc + 4 * (bb * wsp + k))
        acc.append((f"B7 transpose read e0={e0}", "ds_read_b128", addr, 4))
    # B1 gathered partial stores (polling waves 4-5): float4 per unit quad
    JQ = J // 4
    n16 = NG * BC * JQ
    GLK = (80 * BC + 64 * 2 - 1) // (64 * 2)
    for pw in range(2 if old else 0):
        for g in range(GLK):
            addr = []
            for l in range(64):
                idx = l + 64 * (g * 2 + pw)
                if idx >= n16:
                    addr.append(None)
                    continue
                pb, qd = idx // JQ, idx % JQ
                addr.append(sdh + 4 * (pb * J + 4 * qd))
            acc.append((f"B1 partial store wave {4 + pw} sweep {g}", "ds_write_b128", addr, 1))
    if not old:  # round 4: one 16-B store per (slot, b, quad) lane, BSL_G = 3 slot groups per wave
        for pw in range(2):
            addr = []
            for l in range(64):
                gi, bq = l // (5 * BC), l % (5 * BC)
                b, qd, sl = bq // 5, bq % 5, pw * 3 + gi
                ok = gi < 3 and sl < BSL_N and qd < J // 4 and b < BC
                addr.append(sdh + 4 * ((sl * BC + b) * J + 4 * qd) if ok else None)
            acc.append((f"B1 slot partial store wave {4 + pw}", "ds_write_b128", addr, 1))
    # B8 prefetch commit (waves 6-7): round 2 / 3 straight into the record; round 4 into a
    # wave-private slot-major staging block, then one lane per cell writes its factor record (2 x 16 B)
    NPF = 128
    nsl = 7 if cell == "lstm" else 6
    ncell = BC * J
    cpw, cpwp = (ncell + 1) // 2, (BC * 20 + 1) // 2
    NQ = (BC * 20 * 8 + NPF - 1) // NPF if old else (nsl * cpwp + 63) // 64
    for wv in (6, 7):
        for q in range(NQ):
            addr = []
            for l in range(64):
                if old:
                    i = (wv - 6) * 64 + l + q * NPF
                    slot, c = i // (BC * J), i % (BC * J)
                    ok = slot < 8 and c < BC * J
                    dst = ((c // J) * 32 + c % J) * 8 + slot
                else:
                    i = l + 64 * q
                    slot, c = i // cpw, i % cpw
                    ok = slot < nsl and (wv - 6) * cpw + c < ncell
                    dst = 2 * 2 * (BC * 32 * 4 + 16) + (wv - 6) * nsl * cpwp + slot * cpwp + c
                addr.append(sop + 4 * dst if ok else None)
            acc.append((f"B8 prefetch commit wave {wv} q={q}", "ds_write_b32", addr, 1))
        if not old:
            for k in range(nsl):
                addr = [sop + 4 * (2 * 2 * (BC * 32 * 4 + 16) + (wv - 6) * nsl * cpwp + k * cpwp + l)
                        if l < cpw else None for l in range(64)]
                acc.append((f"B9 staging read {k} wave {wv}", "ds_read_b32", addr, 1))
            for pl in range(2):
                addr = [sop + 4 * (pl * (BC * 32 * 4 + 16) + ((wv - 6) * cpw + l) * 4) if l < cpw else None
                        for l in range(64)]
                acc.append((f"B9 factor record store {pl} wave {wv}", "ds_write_b128", addr, 1))
    return acc


def report(name, acc, verbose):
    tot = extra = 0
    for what, ins, addr, mult in acc:
        c, m = cycles(ins, addr)
        tot += c * mult
        extra += (c - m) * mult
        if verbose and c > m:
            print(f"  {what:48s} {ins:14s} x{mult:g}: {c} cycles (min {m})")
    print(f"{name}: {tot:g} LDS-array cycles per step per workgroup, {extra:g} conflict cycles "
          f"({extra / max(tot, 1):.2f})")
    return tot, extra


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--old", action="store_true")
    ap.add_argument("-q", action="store_true")
    a = ap.parse_args()
    v = not a.q
    report("fwd LSTM", fwd_accesses("lstm", a.old), v)
    report("fwd LSTM + fused projection (XK=20 B reads)", fwd_accesses("lstm", a.old, XW=True) + xw_accesses(a.old), v)
    report("fwd LSTM + fused projection (XK=5 B reads)", fwd_accesses("lstm", a.old, XW=True) + xw_accesses(a.old, XK=5),
           v)
    report("fwd LSTM + fused projection, round-3 xfinal layout",
           fwd_accesses("lstm", a.old, XW=True) + xw_accesses(a.old, xfinal_layout="r3"), v)
    report("bwd LSTM", bwd_accesses("lstm", a.old), v)
    report("fwd GRU", fwd_accesses("gru", a.old), v)
    report("bwd GRU", bwd_accesses("gru", a.old), v)


if __name__ == "__main__":
    main()
