"""Write profiles/<name>.json from a tools/pmc_profile.sh directory: per-launch mean counters of the
Strong sweep kernel and the HBM traffic estimate bench.py reports as roofline.traffic.
    python tools/pmc_json.py gpurun_out/pmcNN profiles/r1_pmc_sweep_strong.json [kernel_stats.csv]
HBM bytes per launch = 2 x FETCH_SIZE (gfx950 reports half of wide reads, MI355X_MICROARCH.md §HBM)
+ WRITE_SIZE, both in KiB from rocprofv3; the per-width calibration of narrow gathers is open."""
import csv, glob, json, os, sys, collections
src, dst = sys.argv[1], sys.argv[2]
d = collections.defaultdict(list)
name = None
for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "k_sweep_strong" not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"]
        per[(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (k, _), v in per.items():
        d[k].append(v)
m = {k: sum(v) / len(v) for k, v in d.items()}
out = {"kernel": "k_sweep_strong", "kernel_symbol": name, "width": 3024, "height": 2016, "n_src": 8,
       "counters_per_launch": {k: round(v, 1) for k, v in sorted(m.items())}}
if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
    out["fetch_bytes_raw"] = m["FETCH_SIZE"] * 1024
    out["write_bytes"] = m["WRITE_SIZE"] * 1024
    out["hbm_bytes_per_launch"] = 2 * m["FETCH_SIZE"] * 1024 + m["WRITE_SIZE"] * 1024
    out["correction"] = "2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes); narrow-gather widths uncalibrated"
if "SQ_WAVE_CYCLES" in m:
    w = m["SQ_WAVE_CYCLES"]
    out["derived"] = {"wait_frac": m["SQ_WAIT_ANY"] / w, "issue_stall_frac": m["SQ_WAIT_INST_ANY"] / w,
                      "active_frac": m["SQ_ACTIVE_INST_ANY"] / w,
                      "valu_per_wave": m["SQ_INSTS_VALU"] / m["SQ_WAVES"],
                      "l2_hit": m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]) if "TCC_HIT_sum" in m else None,
                      "l1_miss_req_per_gather": m["TCP_TCC_READ_REQ_sum"] / m["SQ_INSTS_VMEM_RD"] if "TCP_TCC_READ_REQ_sum" in m else None}
if len(sys.argv) > 3:
    for r in csv.DictReader(open(sys.argv[3])):
        if "k_sweep_strong" in r["Name"]:
            out["rocprof_avg_launch_ns"] = float(r["AverageNs"])
out["source"] = "rocprofv3 --pmc, one pass per counter group (tools/pmc_profile.sh), bench.py --steps 2 --warmup 1"
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
