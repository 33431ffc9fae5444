"""Per-kernel register, scratch (private_segment_fixed_size), occupancy and static LDS of the gfx950
code objects, from the compiler's kernel-resource-usage remarks (no GPU needed):
    python3 tools/resource_usage.py > profiles/r6_resource_usage.txt"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         "--cuda-device-only", "-c", "-o", "/tmp/apd_ru.o", "-Rpass-analysis=kernel-resource-usage"]
KEYS = [("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("sgpr", r"SGPRs: (\d+)"),
        ("scratch_B_per_lane", r"ScratchSize \[bytes/lane\]: (\d+)"), ("waves_per_simd", r"Occupancy \[waves/SIMD\]: (\d+)"),
        ("static_lds_B", r"LDS Size \[bytes/block\]: (\d+)")]
for src in ("apde-mvs_amd/csrc/apd_kernels.hip", "apde-mvs_amd/csrc/apd_fusion.hip"):
    r = subprocess.run(["/opt/rocm/bin/hipcc"] + FLAGS + [os.path.join(REPO, src)], capture_output=True, text=True)
    if r.returncode != 0:
        sys.exit(r.stderr[-2000:])
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        for k, pat in KEYS:
            m = re.search(pat, line)
            if m and cur is not None:
                cur[k] = int(m.group(1))
    print(f"# {src}")
    for row in rows:
        name = subprocess.run(["c++filt", row["name"]], capture_output=True, text=True).stdout.strip()
        print(f"{name[:100]:100s} " + " ".join(f"{k} {row.get(k)}" for k, _ in KEYS))
