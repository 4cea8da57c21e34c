"""Spans of the pseudo-inverse forward chains in a rocprofv3 kernel trace.

    python scripts/chain_summary.py <dir with *kernel_trace.csv> [--after sim2_softmax_kernel] [--n 14]

A chain = the `n` consecutive pinv_stage_kernel dispatches that follow each dispatch of the
`after` kernel (tm_pinv_fwd_split is called right after tm_nys_sim2_softmax_split).  Prints the
mean span (first start -> last end), the mean per-launch duration and the mean gap between
launches, i.e. what bench.py's roofline.kernel_ms (HIP events around the call) measures.
"""
import argparse
import csv
import glob
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--after", default="sim2_softmax_kernel")
    ap.add_argument("--kernel", default="pinv_stage_kernel")
    ap.add_argument("--n", type=int, default=14)
    ap.add_argument("--fetch", default="", help="PMC pass dir with FETCH_SIZE (adds the chain's HBM bytes)")
    ap.add_argument("--write", default="", help="PMC pass dir with WRITE_SIZE")
    a = ap.parse_args()
    rows = []
    for f in glob.glob(f"{a.root}/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    if not rows:  # a PMC pass directory: one row per dispatch and counter
        seen = set()
        for f in glob.glob(f"{a.root}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Dispatch_Id"] not in seen:
                    seen.add(r["Dispatch_Id"])
                    rows.append(r)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    spans, durs, gaps, chains = [], [], [], []
    i = 0
    while i < len(rows):
        if a.after in rows[i]["Kernel_Name"]:
            chain = rows[i + 1:i + 1 + a.n]
            if len(chain) == a.n and all(a.kernel in r["Kernel_Name"] for r in chain):
                st = [int(r["Start_Timestamp"]) for r in chain]
                en = [int(r["End_Timestamp"]) for r in chain]
                spans.append((en[-1] - st[0]) / 1e3)
                durs += [(e - s) / 1e3 for s, e in zip(st, en)]
                gaps += [(st[k + 1] - en[k]) / 1e3 for k in range(a.n - 1)]
                chains.append([r["Dispatch_Id"] for r in chain])
                i += a.n
        i += 1
    res = dict(chains=len(spans), launches_per_chain=a.n,
               span_us_mean=round(statistics.mean(spans), 3) if spans else None,
               span_us_median=round(statistics.median(spans), 3) if spans else None,
               launch_us_mean=round(statistics.mean(durs), 3) if durs else None,
               gap_us_mean=round(statistics.mean(gaps), 3) if gaps else None)
    if a.fetch and a.write and chains:
        def per_dispatch(d, counter):
            out = {}
            for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
                for r in csv.DictReader(open(f)):
                    if r["Counter_Name"] == counter:
                        out[r["Dispatch_Id"]] = float(r["Counter_Value"])
            return out
        fe, wr = per_dispatch(a.fetch, "FETCH_SIZE"), per_dispatch(a.write, "WRITE_SIZE")
        # the three PMC runs are separate processes with the same dispatch order: chains found in
        # the FETCH run index both (ids are per run)
        tot = []
        for ids in chains:
            if all(i in fe and i in wr for i in ids):
                tot.append(sum(2 * fe[i] * 1024 + wr[i] * 1024 for i in ids))
        if tot:
            res["traffic_bytes_per_chain"] = round(statistics.mean(tot))
            res["traffic_note"] = "FETCH_SIZE x2 (gfx950 half-count of 16-B reads) + WRITE_SIZE, KiB -> B"
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
