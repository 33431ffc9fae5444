"""Summarise tools/fetch_calib.sh: per calibration kernel the bytes FETCH_SIZE counts per 128-B line it
reads from HBM, the raw fabric read requests, and the time. Usage: python tools/fetch_calib_summary.py OUTDIR"""
import collections, csv, glob, json, os, statistics, sys
out = sys.argv[1]
LINES = (1 << 30) // 128
ms = collections.defaultdict(list)
for l in open(os.path.join(out, "timing.jsonl")):
    r = json.loads(l)
    if r["rep"] > 0:
        ms[r["kernel"]].append(r["ms"])
cnt = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].strip()
        cnt[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {}
for k in ("k_stream16", "k_line_dword", "k_line_dwordx2", "k_line_2x64", "k_line_half"):
    c = {n: statistics.median(v) for n, v in cnt.get(k, {}).items()}
    r = {"ms": round(statistics.median(ms[k]), 4) if ms.get(k) else None}
    true_bytes = 1 << 30  # every kernel reads all 2^23 lines of the 1 GiB buffer once
    r["true_bytes_if_whole_lines"] = true_bytes
    if "FETCH_SIZE" in c:
        fb = c["FETCH_SIZE"] * 1024
        r["fetch_size_bytes"] = fb
        r["fetch_bytes_per_line"] = round(fb / LINES, 2)
        r["factor_whole_lines"] = round(true_bytes / fb, 3)
    for n in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum"):
        if n in c:
            r[n + "_per_line"] = round(c[n] / LINES, 3)
    if r["ms"]:
        r["gbs_if_whole_lines"] = round(true_bytes / (r["ms"] * 1e-3) / 1e9, 1)
    res[k] = r
print(json.dumps(res, indent=1))
