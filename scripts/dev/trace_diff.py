"""Per-kernel time per step of rocprofv3 kernel traces, A runs vs B runs (each side: the minimum
over its runs of the per-step mean, so clock drift between runs counts against neither), matched
by name, over the middle half of the timed graph replays (steps found by a marker kernel).
    python scripts/dev/trace_diff.py "gpurun_out/prof_A*" "gpurun_out/prof_B*" [marker]"""
import csv, glob, sys, collections


def load(path, marker):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    idx = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    idx = idx[len(idx) // 4: 3 * len(idx) // 4]
    per = collections.defaultdict(float); cnt = collections.defaultdict(int)
    for a, b in zip(idx[:-1], idx[1:]):
        for r in rows[a:b]:
            n = r['Kernel_Name'].replace('(anonymous namespace)::', '')[:70]
            per[n] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
            cnt[n] += 1
    k = max(len(idx) - 1, 1)
    return {n: (per[n] / k, cnt[n] / k) for n in per}


def side(pattern, marker):
    runs = [load(f, marker) for f in sorted(glob.glob(pattern + "/run_kernel_trace.csv"))]
    out = {}
    for r in runs:
        for n, v in r.items():
            out[n] = min(out.get(n, v), v, key=lambda t: t[0])
    return out, len(runs)


marker = sys.argv[3] if len(sys.argv) > 3 else 'head_ce_fwd'
A, na = side(sys.argv[1], marker)
B, nb = side(sys.argv[2], marker)
names = sorted(set(A) | set(B), key=lambda n: -max(A.get(n, (0, 0))[0], B.get(n, (0, 0))[0]))
print(f"{'A us':>8} {'B us':>8} {'diff':>7}  kernel (calls A/B)   [{na} A runs, {nb} B runs]")
for n in names:
    a, ca = A.get(n, (0, 0)); b, cb = B.get(n, (0, 0))
    if max(a, b) < 0.5: continue
    print(f"{a:8.1f} {b:8.1f} {a - b:7.1f}  {n} ({ca:.0f}/{cb:.0f})")
print(f"{sum(v[0] for v in A.values()):8.1f} {sum(v[0] for v in B.values()):8.1f}  total per step")
