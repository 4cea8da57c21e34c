"""Per-launch HBM bytes of selected kernels from two rocprofv3 --pmc passes.

    python scripts/traffic_summary.py <fetch_dir> <write_dir> <kernel substring>...

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE counts exactly
half the bytes of a wide (16 B per lane) coalesced read (MI355X_MICROARCH.md, HBM), so
the read side is doubled; WRITE_SIZE is exact for 16-B stores.  Prints one JSON object.
"""
import csv
import glob
import json
import sys


def collect(d, counter, keys):
    files = glob.glob(f"{d}/**/*counter_collection*.csv", recursive=True)
    out = {k: [] for k in keys}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r.get("Kernel_Name", "")
            for k in keys:
                if k in name:
                    out[k].append(float(r["Counter_Value"]))
    return out


def main():
    fdir, wdir, keys = sys.argv[1], sys.argv[2], sys.argv[3:]
    fe = collect(fdir, "FETCH_SIZE", keys)
    wr = collect(wdir, "WRITE_SIZE", keys)
    res = {}
    for k in keys:
        if not fe[k] or not wr[k]:
            res[k] = None
            continue
        f = sum(fe[k]) / len(fe[k]) * 1024
        w = sum(wr[k]) / len(wr[k]) * 1024
        res[k] = dict(fetch_size_bytes=f, write_size_bytes=w, read_bytes_corrected=2 * f,
                      traffic_bytes=2 * f + w, dispatches=[len(fe[k]), len(wr[k])])
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
