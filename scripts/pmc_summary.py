"""Per-kernel PMC summary of the passes written by scripts/gpu_pmc_bench.sh.

    python scripts/pmc_summary.py gpurun_out/pmc [--top 12] [--kernels a,b,...]

For every kernel: dispatches, mean duration (from the kernel trace of the SQ pass), and per
dispatch: HBM bytes (FETCH_SIZE doubled for the gfx950 half-count of 16-B reads + WRITE_SIZE,
MI355X_MICROARCH.md "HBM"), L2 hit rate, MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES /
(dispatch cycles x 1024 SIMDs), CU busy = SQ_BUSY_CU_CYCLES / (dispatch cycles x 256 CUs), with
dispatch cycles = duration x CLOCK_GHZ (rocprofv3's MfmaUtil divides by GRBM_GUI_ACTIVE, which
reads high on short dispatches), wave-cycle shares (wait / issue-stall /
active; SQ_WAVE_CYCLES counts quad-cycles like the SQ_WAIT_* counters), and the effective clock
GRBM_GUI_ACTIVE / 8 XCDs / duration.  Prints one JSON object.
"""
import argparse
import collections
import csv
import glob
import json
import re

CLOCK_GHZ = 2.0   # in-kernel shader clock under load (s_memtime vs s_memrealtime stamps, pinv stage)


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*$", "", name) if not name.startswith("void ") else re.sub(r"\(.*$", "", name[5:])
    return name.strip()


def counters(d):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection*.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            out[short(r.get("Kernel_Name", ""))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def durations(d):
    out = collections.defaultdict(list)
    for f in glob.glob(f"{d}/**/*kernel_trace*.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            out[short(r["Kernel_Name"])].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
    return out


def mean(v):
    return sum(v) / len(v) if v else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--top", type=int, default=14)
    ap.add_argument("--kernels", default="")
    a = ap.parse_args()
    c = collections.defaultdict(dict)
    for p in ("sq", "tcc", "fetch", "write", "lds"):
        for k, cs in counters(f"{a.root}/{p}").items():
            for n, v in cs.items():
                c[k][n] = v
    dur = durations(f"{a.root}/sq") or durations(f"{a.root}/fetch")
    total = {k: sum(v) for k, v in dur.items()}
    names = sorted(total, key=lambda k: -total[k])
    if a.kernels:
        names = [k for k in names if any(s in k for s in a.kernels.split(","))]
    res = {}
    for k in names[:a.top]:
        cs = c.get(k, {})
        m = {n: mean(v) for n, v in cs.items()}
        t = mean(dur[k])
        row = dict(dispatches=len(dur[k]), mean_us=round(t / 1e3, 3), share=round(total[k] / sum(total.values()), 4))
        if m.get("FETCH_SIZE") is not None and m.get("WRITE_SIZE") is not None:
            row["hbm_bytes"] = round(2 * m["FETCH_SIZE"] * 1024 + m["WRITE_SIZE"] * 1024)
            row["hbm_GBps"] = round(row["hbm_bytes"] / t, 1)
        if m.get("TCC_HIT_sum") is not None:
            h, mi = m["TCC_HIT_sum"], m["TCC_MISS_sum"]
            row["l2_hit"] = round(h / max(h + mi, 1), 3)
        # GRBM_GUI_ACTIVE / 8 reads high on dispatches shorter than ~0.3 ms (MI355X_MICROARCH.md,
        # DVFS give-back), so the busy fractions use the in-kernel clock measured by s_memtime /
        # s_memrealtime stamps (CLOCK_GHZ) x the dispatch duration
        cyc = t * CLOCK_GHZ  # t in ns
        if m.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
            row["mfma_busy_cycles"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"])
            row["mfma_util"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024), 4)
        if m.get("SQ_BUSY_CU_CYCLES") is not None:
            row["cu_busy"] = round(m["SQ_BUSY_CU_CYCLES"] / (cyc * 256), 4)
        if m.get("SQ_WAVE_CYCLES"):
            w = m["SQ_WAVE_CYCLES"]
            row["wait_any"] = round(m["SQ_WAIT_ANY"] / w, 3)
            row["wait_inst_any"] = round(m["SQ_WAIT_INST_ANY"] / w, 3)
            row["active_inst_any"] = round(m["SQ_ACTIVE_INST_ANY"] / w, 3)
        if m.get("GRBM_GUI_ACTIVE"):
            row["clock_GHz"] = round(m["GRBM_GUI_ACTIVE"] / 8 / t, 3)
        for n in ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS",
                  "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
            if m.get(n) is not None:
                row[n] = m[n]
        row["raw"] = {n: v for n, v in m.items()}
        res[k] = row
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
