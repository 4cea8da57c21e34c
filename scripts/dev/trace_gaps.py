"""Kernel-boundary gaps of the bench's graph replay from a rocprofv3 kernel trace: for every kernel
(by name), its average duration and the average idle gap between its end and the next kernel's
start on the same queue (the dependent-launch boundary it leaves behind: launch + the L2 write-back
of what it left dirty, MI355X_MICROARCH.md price list, row 'boundary').

    python scripts/dev/trace_gaps.py <kernel_trace.csv> [--min-gap-us 0] [--steps-window 200]
"""
import argparse
import csv
import collections


def short(name, width=70):
    name = name.replace("void ", "")
    return name if len(name) <= width else name[:width - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r.get("Queue_Id", r.get("Stream_Id", "0"))))
    rows.sort()
    # the longest run of kernels with no gap above 50 us = the timed graph replays
    runs, cur = [], [rows[0]]
    for a, b in zip(rows, rows[1:]):
        if b[0] - a[1] > 50_000:
            runs.append(cur)
            cur = []
        cur.append(b)
    runs.append(cur)
    run = max(runs, key=len)
    dur = collections.defaultdict(list)
    gap_after = collections.defaultdict(list)
    for a, b in zip(run, run[1:]):
        dur[a[2]].append((a[1] - a[0]) / 1e3)
        gap_after[a[2]].append(max(0, b[0] - a[1]) / 1e3)
    total_span = (run[-1][1] - run[0][0]) / 1e3
    busy = sum(sum(v) for v in dur.values())
    gaps = sum(sum(v) for v in gap_after.values())
    print(f"window: {len(run)} kernels over {total_span:.1f} us: busy {busy:.1f} us, gaps {gaps:.1f} us")
    spin = [k for k in dur if "spin_kernel" in k]
    order = sorted(gap_after, key=lambda k: -sum(gap_after[k]))
    print(f"{'kernel':70s} {'calls':>6} {'dur us':>8} {'gap us':>8} {'gap tot':>8}")
    for k in order[:args.top]:
        if k in spin:
            continue
        n = len(gap_after[k])
        print(f"{short(k):70s} {n:6d} {sum(dur[k]) / n:8.2f} {sum(gap_after[k]) / n:8.2f} {sum(gap_after[k]):8.1f}")


if __name__ == "__main__":
    main()
