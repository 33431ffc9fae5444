"""Write profiles/<name>.json from a tools/pmc_profile.sh / tools/pmc_c3.sh directory: per-launch mean
counters of one kernel and the HBM traffic estimate bench.py reports as roofline.traffic.
    python tools/pmc_json.py <pmc dir> <out.json> [--kernel k_sweep_strong] [--width 3024 --height 2016
                             --n-src 8] [--stats kernel_stats.csv] [--source "..."]
HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE, both in KiB from rocprofv3: gfx950 tallies each
128-B line fill as one 64-B request for every access width these kernels use (4-, 8- and 16-byte
loads, one or both line halves: profiles/r5_fetch_calibration.json, tools/fetch_calib.hip)."""
import argparse, csv, glob, json, os, collections
ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("dst")
ap.add_argument("--kernel", default="k_sweep_strong")
ap.add_argument("--width", type=int, default=3024)
ap.add_argument("--height", type=int, default=2016)
ap.add_argument("--n-src", type=int, default=8)
ap.add_argument("--stats")
ap.add_argument("--last", type=int, default=0, help="only the last N dispatches of the kernel (e.g. the APD pass after its FIRST_INIT priors)")
ap.add_argument("--source-hash", help="kernel-source hash of the profiled build (default: <src>/source_hash, "
                                      "written by tools/pmc_c3.sh at collection time)")
ap.add_argument("--source", default="rocprofv3 --pmc, one pass per counter group (tools/pmc_profile.sh), "
                                    "bench.py --steps 2 --warmup 1")
a = ap.parse_args()
d = collections.defaultdict(list)
name = None
for f in glob.glob(os.path.join(a.src, "**", "*counter_collection.csv"), recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if a.kernel not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"]
        per[(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    if a.last > 0:
        keep = sorted({int(i) for (_, i) in per}, reverse=False)[-a.last:]
        per = {k: v for k, v in per.items() if int(k[1]) in keep}
    for (k, _), v in per.items():
        d[k].append(v)
m = {k: sum(v) / len(v) for k, v in d.items()}
out = {"kernel": a.kernel, "kernel_symbol": name, "width": a.width, "height": a.height, "n_src": a.n_src,
       "launches_sampled": max((len(v) for v in d.values()), default=0),
       "counters_per_launch": {k: round(v, 1) for k, v in sorted(m.items())}}
if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
    out["fetch_bytes_raw"] = m["FETCH_SIZE"] * 1024
    out["write_bytes"] = m["WRITE_SIZE"] * 1024
    out["hbm_bytes_per_launch"] = 2 * m["FETCH_SIZE"] * 1024 + m["WRITE_SIZE"] * 1024
    out["correction"] = "2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes)"
    out["correction_factor"] = 2.0
    out["correction_calibration"] = "profiles/r5_fetch_calibration.json"
if "SQ_WAVE_CYCLES" in m:
    w = m["SQ_WAVE_CYCLES"]
    g = lambda k: m.get(k)
    out["derived"] = {"wait_frac": g("SQ_WAIT_ANY") / w if g("SQ_WAIT_ANY") else None,
                      "issue_stall_frac": g("SQ_WAIT_INST_ANY") / w if g("SQ_WAIT_INST_ANY") else None,
                      "active_frac": g("SQ_ACTIVE_INST_ANY") / w if g("SQ_ACTIVE_INST_ANY") else None,
                      "valu_per_wave": m["SQ_INSTS_VALU"] / m["SQ_WAVES"] if "SQ_INSTS_VALU" in m else None,
                      "valu_per_gather": m["SQ_INSTS_VALU"] / m["SQ_INSTS_VMEM_RD"] if "SQ_INSTS_VMEM_RD" in m else None,
                      "l2_hit": m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]) if "TCC_HIT_sum" in m else None,
                      "l1_miss_req_per_gather": m["TCP_TCC_READ_REQ_sum"] / m["SQ_INSTS_VMEM_RD"]
                      if "TCP_TCC_READ_REQ_sum" in m and "SQ_INSTS_VMEM_RD" in m else None,
                      "l1_miss_frac": m["TCP_TCC_READ_REQ_sum"] / m["TCP_TOTAL_CACHE_ACCESSES_sum"]
                      if "TCP_TOTAL_CACHE_ACCESSES_sum" in m and "TCP_TCC_READ_REQ_sum" in m else None}
if a.stats:
    for r in csv.DictReader(open(a.stats)):
        if a.kernel in r["Name"]:
            out["rocprof_avg_launch_ns"] = float(r["AverageNs"])
sh = a.source_hash
if sh is None and os.path.exists(os.path.join(a.src, "source_hash")):
    sh = open(os.path.join(a.src, "source_hash")).read().strip()
out["source_hash"] = sh  # bench.py latest_pmc reports this summary only while it equals bench.source_hash()
out["source"] = a.source
json.dump(out, open(a.dst, "w"), indent=1)
print(json.dumps(out, indent=1))
