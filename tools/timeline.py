"""Per-kernel timeline of one training step from a rocprofv3 kernel trace.

  python tools/timeline.py <kernel_trace.csv> [step index from the end, default 1]

Prints every dispatch between a step's mixing kernel (source_stats_kernel) and its Adam
(adam_kernel): start offset and duration in us, and the queue it ran on -- to see what
overlaps (side streams) and where the step's critical path is."""
import csv
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(")[0] if not name.startswith("void ") else name[5:].split("(")[0]


def main(path, back=1):
    rows = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r.get("Queue_Id", r.get("Stream_Id", "?")), r.get("Grid_Size", r.get("Grid_Size_X", "?")))
            for r in csv.DictReader(open(path))]
    rows.sort(key=lambda r: r[1])
    starts = [r[1] for r in rows if r[0] == "source_stats_kernel"]
    ends = [r[2] for r in rows if r[0].startswith("adam_kernel")]
    t0 = starts[-back]
    t1 = min(e for e in ends if e > t0)
    print(f"step: {(t1 - t0) / 1e3:.1f} us")
    for nm, a, b, q, gsz in rows:
        if a >= t0 and b <= t1:
            print(f"{(a - t0) / 1e3:9.1f} {(b - a) / 1e3:8.1f}  q{q:<3} grid {gsz:<8} {nm[:80]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
