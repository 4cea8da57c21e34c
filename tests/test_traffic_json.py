"""scripts/traffic_json.py (profiles/traffic.json from rocprofv3 PMC passes) on a synthetic pass
directory: per-site bytes = 2 x FETCH_SIZE + WRITE_SIZE per dispatch, two-layer sites split by
dispatch order, the pinv forward chain = the 14 pinv_stage dispatches after each A3 forward."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(d, counter, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, (name, kib) in enumerate(rows):
            w.writerow(dict(Dispatch_Id=i, Kernel_Name=name, Counter_Name=counter, Counter_Value=kib))


def test_traffic_json_sites(tmp_path):
    step = [("_ZN12_GLOBAL__N_113ln_fwd_kernelIDF16bLi8EEEvPKf(float)", 10.0),
            ("void a3_fwd_v2_kernel<0, 4>(float const*)", 100.0)]
    step += [("void pinv_stage_kernel<false>(SLaunch)", 1.0)] * 13 + [("void pinv_stage_kernel<true>(SLaunch)", 3.0)]
    step += [("_ZN12_GLOBAL__N_113ln_fwd_kernelIDF16bLi8EEEvPKf(float)", 20.0),
             ("void a3_fwd_v2_kernel<0, 4>(float const*)", 200.0)]
    step += [("void pinv_stage_kernel<false>(SLaunch)", 1.0)] * 13 + [("void pinv_stage_kernel<true>(SLaunch)", 3.0)]
    _write(tmp_path / "fetch", "FETCH_SIZE", step * 2)
    _write(tmp_path / "write", "WRITE_SIZE", [(n, v / 2) for n, v in step * 2])
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "traffic_json.py"), str(tmp_path),
                          "--commit", "test", "--n", "8192"], capture_output=True, text=True, cwd=ROOT, check=True)
    sites = json.loads(out.stdout)["sites"]
    kib = 1024
    assert sites["ln_fwd:1"]["traffic_bytes"] == int((2 * 10 + 5) * kib)
    assert sites["ln_fwd:2"]["traffic_bytes"] == int((2 * 20 + 10) * kib)
    assert sites["a3_fwd:2"]["traffic_bytes"] == int((2 * 200 + 100) * kib)
    assert sites["pinv_fwd"]["traffic_bytes"] == int((2 * 16 + 8) * kib)
    assert sites["pinv_fwd"]["dispatches"] == [4, 4]
    assert sites["ln_fwd:1"]["algorithmic_bytes"] > 0


def test_committed_traffic_reaches_the_bench_on_the_gpu_box():
    """bench.py's roofline.traffic reads profiles/traffic.json at run time on the GPU box: the file
    must be committed for the bench workload and must not be excluded from the gpurun snapshot
    (.gpurunignore patterns are tar excludes; an exclude of the whole profiles/ directory made the
    round-3 / early round-4 bench lines carry traffic: null)."""
    import fnmatch
    sys.path.insert(0, ROOT)
    import bench
    rec = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))["sites"]
    for site in ("pinv_fwd", "pinv_bwd", "ln_fwd:1", "a3_bwd:1"):
        assert bench.measured_traffic(site, 8192, "bf16") == rec[site]["traffic_bytes"] > 0
    pats = [l.strip() for l in open(os.path.join(ROOT, ".gpurunignore")) if l.strip() and not l.startswith("#")]
    member = "./profiles/traffic.json"
    for p in pats:
        anchored = p.startswith("./")
        hit = fnmatch.fnmatch(member, p) if anchored else fnmatch.fnmatch(os.path.basename(member), p)
        hit = hit or (anchored and member.startswith(p.rstrip("/") + "/"))
        assert not hit, f".gpurunignore pattern {p!r} drops {member}"
