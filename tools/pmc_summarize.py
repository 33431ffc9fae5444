"""Summarise tools/pmc_profile.sh output: per-dispatch mean of each counter for one kernel.
    python tools/pmc_summarize.py gpurun_out/pmc [kernel-substring]"""
import csv, glob, json, os, sys
from collections import defaultdict

out = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "k_sweep_strong"
vals = defaultdict(list)
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    per = defaultdict(float)
    for row in csv.DictReader(open(f)):
        if sub not in row["Kernel_Name"]:
            continue
        per[(row["Counter_Name"], row["Dispatch_Id"])] += float(row["Counter_Value"])
    for (name, _), v in per.items():
        vals[name].append(v)
res = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
print(json.dumps(res, indent=1))
w = res.get("SQ_WAVE_CYCLES")
if w:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
        if k in res:
            print(f"{k}/WAVE_CYCLES = {res[k] / w:.3f}")
if "SQ_WAVES" in res:
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
        if k in res:
            print(f"{k}/wave = {res[k] / res['SQ_WAVES']:.0f}")
if "TCC_HIT_sum" in res:
    print("L2 hit", res["TCC_HIT_sum"] / (res["TCC_HIT_sum"] + res["TCC_MISS_sum"]))
if "TCP_TCC_READ_REQ_sum" in res and "SQ_INSTS_VMEM_RD" in res:
    print("L2 req / VMEM rd instr", res["TCP_TCC_READ_REQ_sum"] / res["SQ_INSTS_VMEM_RD"])
