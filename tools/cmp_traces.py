"""Per-kernel time per training step (us) of several kernel traces (tools/trace_multi.sh): the steps are
source_stats_kernel start .. the following adam_kernel end, the first two skipped (graph capture)."""
import collections
import csv
import sys


def load(p):
    rows = [(r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", ""),
             int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(p))]
    rows.sort(key=lambda r: r[1])
    starts = [r[1] for r in rows if r[0].startswith("source_stats_kernel")]
    ends = [r[2] for r in rows if r[0].startswith("adam_kernel")]
    acc, spans, bwd = collections.defaultdict(float), [], []
    for t0 in starts[2:]:
        e = [x for x in ends if x > t0]
        if not e:
            break
        t1 = min(e)
        spans.append((t1 - t0) / 1e3)
        for nm, a, b in rows:
            if a >= t0 and b <= t1:
                k = nm.split("(")[0][:70]
                k = k.replace("Cfg<256, 3>", "Cfg<256, 3, 64>").replace("Cfg<128, 2>", "Cfg<128, 2, 64>")
                acc[k] += (b - a) / 1e3
                if k.startswith("rnn_bwd"):
                    bwd.append((b - a) / 1e3)
    n = len(spans)
    return {k: v / n for k, v in acc.items()}, spans, [sum(bwd[i::4]) / n for i in range(4)]


base = sys.argv[1]
tags = sys.argv[2:]
res = {t: load(f"{base}/{t}/run_kernel_trace.csv") for t in tags}
for t in tags:
    k, sp, bw = res[t]
    print(f"{t:10s} step span {sum(sp[1:]) / len(sp[1:]):7.1f} us  bwd launches", [round(x, 1) for x in bw],
          "fwd", round(sum(v for kk, v in k.items() if kk.startswith("rnn_fwd")), 1))
keys = sorted(set().union(*[set(r[0]) for r in res.values()]), key=lambda k: -res[tags[0]][0].get(k, 0))
print(f"{'kernel':70s}" + "".join(f"{t:>10s}" for t in tags))
for k in keys:
    vals = [res[t][0].get(k, 0.0) for t in tags]
    if max(vals) > 2:
        print(f"{k:70s}" + "".join(f"{v:10.1f}" for v in vals))
