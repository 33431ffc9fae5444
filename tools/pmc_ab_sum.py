"""Summarise tools/pmc_ab.sh: per-variant mean counter values per dispatch."""
import csv, glob, os, sys, collections
out = sys.argv[1]
for vdir in sorted(glob.glob(os.path.join(out, "v*"))):
    if not os.path.isdir(vdir):
        continue
    d = collections.defaultdict(list)
    for f in glob.glob(os.path.join(vdir, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            per[(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (k, _), v in per.items():
            d[k].append(v)
    m = {k: sum(v) / len(v) for k, v in d.items()}
    line = {k: f"{v:.3e}" for k, v in sorted(m.items())}
    print(os.path.basename(vdir), line)
    if "SQ_INSTS_VMEM_RD" in m:
        print("   tcp acc/vmem %.1f  l2 req/vmem %.1f" % (m.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0) / m["SQ_INSTS_VMEM_RD"],
                                                          m.get("TCP_TCC_READ_REQ_sum", 0) / m["SQ_INSTS_VMEM_RD"]))
    if "SQ_WAVE_CYCLES" in m:
        w = m["SQ_WAVE_CYCLES"]
        print("   wait %.2f  inst-wait %.2f  active %.2f  valu/wave %.0f" % (m["SQ_WAIT_ANY"] / w, m["SQ_WAIT_INST_ANY"] / w,
              m["SQ_ACTIVE_INST_ANY"] / w, m["SQ_INSTS_VALU"] / m["SQ_WAVES"]))
