"""Summarise one tools/prof_round.sh session into profiles/ (tracked).

  python tools/summarize_prof.py gpurun_out/<TAG> <round-tag> [warmup steps]   (bench's --warmup / --steps)

Writes
  profiles/<round>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<round>_summary.md         per-kernel table (avg us, calls, share) + per-step split
  profiles/<round>_pmc.json           per-kernel HBM traffic per launch from the two PMC passes:
                                      FETCH_SIZE x 2 (gfx950 reports half of wide streaming reads,
                                      MI355X_MICROARCH.md "HBM") + WRITE_SIZE, KB -> bytes
"""
import collections
import csv
import json
import os
import shutil
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0] if not name.startswith("void ") else name[5:].split("(")[0]


def per_step(tr, warmup, steps):
    """Device time per timed step and kernel: the dispatches from the start of step
    warmup+1 (its source_stats_kernel) to the end of step warmup+steps (its adam_kernel),
    so one-off work (warmup, first-call GEMM algorithm timing, the bench's probes) is out."""
    rows = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
            for r in csv.DictReader(open(tr))]
    rows.sort(key=lambda r: r[1])
    starts = [r[1] for r in rows if r[0] == "source_stats_kernel"]
    ends = [r[2] for r in rows if r[0].startswith("adam_kernel")]
    if len(starts) < warmup + steps or len(ends) < warmup + steps:
        return []
    t0, t1 = starts[warmup], ends[warmup + steps - 1]
    acc = collections.defaultdict(float)
    for nm, a, b in rows:
        if a >= t0 and b <= t1:
            acc[nm] += (b - a) / 1e3 / steps
    busy = sum(acc.values())
    out = ["", f"## Per timed step (steps {warmup + 1}..{warmup + steps}: device us per step)", "",
           f"wall {(t1 - t0) / 1e3 / steps:.1f} us per step, kernels busy {busy:.1f} us", "",
           "| kernel | us / step | share % |", "|---|---|---|"]
    for nm, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        out.append(f"| `{nm[:90]}` | {v:.1f} | {100 * v / busy:.1f} |")
    return out


def main(src, tag, out="profiles", warmup=1, steps=3):
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"# {tag}: rocprofv3 --kernel-trace --stats ({src})", "",
             "| kernel | calls | avg us | min us | max us | share % |", "|---|---|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                     f"{float(r['MinNs']) / 1e3:.2f} | {float(r['MaxNs']) / 1e3:.2f} | "
                     f"{100 * float(r['TotalDurationNs']) / tot:.1f} |")
    # per-(kernel, grid) split of the trace: the STFT runs at two sizes in bench.py
    # (in-step launches and the standalone 2048-signal probe)
    tr = os.path.join(src, "trace", "run_kernel_trace.csv")
    if os.path.exists(tr):
        by = collections.defaultdict(list)
        for r in csv.DictReader(open(tr)):
            nm = short(r["Kernel_Name"])
            if "stft" in nm or "gemm" in nm or "rnn" in nm:
                by[(nm, r.get("Grid_Size", r.get("Grid_Size_X", "?")))].append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        lines += ["", "## STFT / GEMM launches by grid size", "", "| kernel | grid | calls | avg us |",
                  "|---|---|---|---|"]
        for (nm, g), v in sorted(by.items()):
            lines.append(f"| `{nm}` | {g} | {len(v)} | {sum(v) / len(v):.2f} |")
        lines += per_step(tr, warmup, steps)
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub, counter in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
        f = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                pmc[short(r["Kernel_Name"])][counter].append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    res = {}
    for k, d in pmc.items():
        fetch = [(g, 2 * 1024 * v) for g, v in d.get("FETCH_SIZE", [])]
        write = [(g, 1024 * v) for g, v in d.get("WRITE_SIZE", [])]
        n = min(len(fetch), len(write))
        if n == 0:
            continue
        # the two passes run the same command: dispatch i of one pass is dispatch i of the other
        per = [{"grid": gf, "fetch": vf, "write": vw, "traffic": vf + vw}
               for (gf, vf), (gw, vw) in zip(fetch[:n], write[:n]) if gf == gw]
        res[k] = {"dispatches": len(per), "launches": per,
                  "avg_traffic_bytes": sum(p["traffic"] for p in per) / max(1, len(per))}
    if res:
        json.dump({"source": src, "correction": "FETCH_SIZE x2 (gfx950), KB->bytes", "kernels": res},
                  open(os.path.join(out, f"{tag}_pmc.json"), "w"), indent=1)
        lines += ["", "## HBM traffic per launch (PMC: FETCH_SIZE x2 + WRITE_SIZE)", "",
                  "| kernel | dispatches | avg MB / launch |", "|---|---|---|"]
        for k, v in sorted(res.items(), key=lambda kv: -kv[1]["avg_traffic_bytes"]):
            lines.append(f"| `{k}` | {v['dispatches']} | {v['avg_traffic_bytes'] / 1e6:.2f} |")
    # MFMA / LDS counter pass (pmc_mfma): per kernel, MFMA-busy fraction of the CU-SIMD cycles
    # the kernel held = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), and
    # LDS bank-conflict cycles as a share of all LDS-array cycles (MI355X_MICROARCH.md §LDS)
    f = os.path.join(src, "pmc_mfma", "run_counter_collection.csv")
    if os.path.exists(f):
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        cnt = collections.defaultdict(int)
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                cnt[k] += 1
        mf = {}
        for k, d in acc.items():
            gui = d.get("GRBM_GUI_ACTIVE", 0.0)
            if gui <= 0:
                continue
            mf[k] = {"dispatches": cnt[k],
                     "mfma_busy_frac": d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui / 8 * 1024),
                     "lds_bank_conflict_frac": d.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, d.get("SQ_LDS_IDX_ACTIVE", 0.0)),
                     "counters": dict(d)}
        json.dump({"source": src, "formula": "MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)", "kernels": mf},
                  open(os.path.join(out, f"{tag}_mfma.json"), "w"), indent=1)
        lines += ["", "## MFMA busy and LDS bank conflicts (PMC pass pmc_mfma)", "",
                  "| kernel | dispatches | MFMA busy | LDS conflict cycles / LDS cycles |", "|---|---|---|---|"]
        for k, v in sorted(mf.items(), key=lambda kv: -kv[1]["counters"].get("SQ_VALU_MFMA_BUSY_CYCLES", 0)):
            if v["counters"].get("SQ_VALU_MFMA_BUSY_CYCLES", 0) > 0:
                lines.append(f"| `{k}` | {v['dispatches']} | {v['mfma_busy_frac']:.3f} | {v['lds_bank_conflict_frac']:.3f} |")
    open(os.path.join(out, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *([] if len(sys.argv) < 5 else ["profiles", int(sys.argv[3]), int(sys.argv[4])]))
