"""profiles/traffic.json from the FETCH_SIZE / WRITE_SIZE passes of scripts/gpu_pmc_bench.sh.

    python scripts/traffic_json.py gpurun_out/pmc --commit <rev> --n 8192 > profiles/traffic.json

HBM bytes per launch of every bench hbm_roofline site (bench.py HBM_SITES) and of the pinv forward
chain (the bench `roofline` kernel): FETCH_SIZE doubled for the gfx950 half-count of 16-B-per-lane
reads (MI355X_MICROARCH.md, HBM) + WRITE_SIZE, per dispatch, mean over the run's dispatches.
Sites with two layers on one kernel are split by dispatch order (forward: layer 1 then 2;
backward: 2 then 1); the pinv forward chain is the 14 pinv_stage dispatches after each
A3 forward dispatch (which also writes A2, the chain's input).  Algorithmic bytes from bench.hbm_model / bench.roofline_model.
"""
import argparse
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    # names the profiler left mangled (a __bf16 parameter defeats its demangler):
    # _ZN12_GLOBAL__N_1<len><identifier>I<template args>... -> the identifier
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)", name)
    if m:
        i = m.end()
        return name[i:i + int(m.group(1))]
    return re.sub(r"\(.*$", "", name).strip()


def dispatches(d, counter):
    """[(dispatch_id, kernel, bytes)] in dispatch order."""
    out = {}
    for f in glob.glob(f"{d}/**/*counter_collection*.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            key = (f, int(r["Dispatch_Id"]))
            out[key] = (short(r["Kernel_Name"]), float(r["Counter_Value"]) * 1024)
    return [(k[1], v[0], v[1]) for k, v in sorted(out.items())]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--commit", required=True)
    ap.add_argument("--n", type=int, default=8192)
    a = ap.parse_args()
    import bench
    fe = dispatches(os.path.join(a.pmc_dir, "fetch"), "FETCH_SIZE")
    wr = dispatches(os.path.join(a.pmc_dir, "write"), "WRITE_SIZE")

    def per_kernel(pat):
        rf = [b for _, k, b in fe if re.search(pat, k)]
        rw = [b for _, k, b in wr if re.search(pat, k)]
        return rf, rw

    def mean(v):
        return sum(v) / len(v) if v else None

    model = bench.hbm_model(a.n, 2)
    sites = {}

    def put(key, pats, layer_of=None, nlayers=1, algo=None, kernel=None):
        tot, disp = 0.0, []
        for pat in pats:
            rf, rw = per_kernel(pat)
            if layer_of is not None:
                rf, rw = rf[layer_of::nlayers], rw[layer_of::nlayers]
            if not rf or not rw:
                return
            tot += 2 * mean(rf) + mean(rw)
            disp.append([len(rf), len(rw)])
        sites[key] = dict(n=a.n, dtype="bf16", kernel=kernel, traffic_bytes=int(tot), algorithmic_bytes=algo,
                          dispatches=disp)

    for site in bench.HBM_SITES:
        layers = bench.SITE_LAYERS[site]
        for k, layer in enumerate(layers):
            if (site, layer) not in model:
                continue
            kname, byts = model[(site, layer)]
            pats = {"ln_fwd": [r"ln_fwd_kernel"], "landmarks": [r"landmarks_kernel"],
                    "a3_fwd": [r"^a3_fwd_v2_kernel"], "a1_fwd": [r"^a1_fwd_bf16_kernel"],
                    "ppeg_fwd": [r"^ppeg_stencil_kernel<false>"],
                    "ppeg_bwd": [r"^ppeg_bwd_kernel"],
                    "conv_bwd": [r"^conv_bwd_mfma_kernel"], "a1_bwd": [r"^attn_bwd_bf16_kernel<1, 8"],
                    "a3_bwd": [r"^attn_bwd_bf16_kernel<0, 9"]}[site]
            key = site if len(layers) == 1 else f"{site}:{layer}"
            put(key, pats, layer_of=k if len(layers) > 1 else None, nlayers=len(layers), algo=byts, kernel=kname)

    # pinv forward chain: the 14 pinv_stage dispatches after each A3 forward (+ A2 rows) dispatch
    def chains(rows):
        out, i = [], 0
        while i < len(rows):
            if rows[i][1].startswith("a3_fwd_v2_kernel") or rows[i][1].startswith("sim2_softmax"):
                seq = [b for _, k, b in rows[i + 1:i + 40] if k.startswith("pinv_stage_kernel")][:14]
                if len(seq) == 14:
                    out.append(sum(seq))
            i += 1
        return out
    cf, cw = chains(fe), chains(wr)
    if cf and cw:
        work = bench.roofline_model("pinv_fwd", a.n, 2)
        sites["pinv_fwd"] = dict(n=a.n, dtype="bf16", kernel="pinv_stage_kernel x14 (tm_pinv_fwd_split_a3)",
                                 traffic_bytes=int(2 * mean(cf) + mean(cw)),
                                 algorithmic_bytes=work.get("bytes"), dispatches=[len(cf), len(cw)])
    # pinv backward: the 24 pinv_stage dispatches before each pinv_apply_bwd_kernel (the last one
    # also computes the c-gradient dot) and the apply itself
    def bwd_chains(rows):
        out = []
        for i, (_, k, b) in enumerate(rows):
            if not k.startswith("pinv_apply_bwd_kernel"):
                continue
            seq = [bb for _, kk, bb in rows[max(0, i - 60):i] if kk.startswith("pinv_stage_kernel")][-24:]
            if len(seq) == 24:
                out.append(sum(seq) + b)
        return out
    bf, bw = bwd_chains(fe), bwd_chains(wr)
    if bf and bw:
        work = bench.roofline_model("pinv_bwd", a.n, 2)
        sites["pinv_bwd"] = dict(n=a.n, dtype="bf16", kernel="pinv_stage_kernel x24 + "
                                 "pinv_apply_bwd_kernel (tm_pinv_bwd_split)",
                                 traffic_bytes=int(2 * mean(bf) + mean(bw)),
                                 algorithmic_bytes=work.get("bytes"), dispatches=[len(bf), len(bw)])
    print(json.dumps(dict(
        note="rocprofv3 --kernel-trace --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
             "`bench.py --steps 3 --warmup 2 --no-cpu-baseline` (scripts/gpu_pmc_bench.sh, PASSES='fetch write'), "
             "summarised by scripts/traffic_json.py: per dispatch, read side doubled for the gfx950 FETCH_SIZE "
             "half-count of 16-B-per-lane reads, WRITE_SIZE as is; includes Infinity-Cache hits (the counters sit "
             "on the L2's fabric side).",
        commit=a.commit, sites=sites), indent=1))


if __name__ == "__main__":
    main()
