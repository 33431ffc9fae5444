"""Whole-scan timing of the `apd` binary (main.cpp's round schedule) on a synthetic scan written as
JPEG images (ETH3D ships JPEG): wall time vs the summed "RunPatchMatch time" lines = host overhead
(decode, resize, file I/O, uploads). Usage (GPU box):
    python tools/time_scan.py [W H VIEWS] [extra apd flags...]
pair.txt lists each view's TIME_SCAN_NSRC (default 10, BASELINE C3's N) nearest views as sources
(0 = all other views). Per pass it reports the loop-body rate (Mpix/s per PatchMatch iteration: W*H*iterations
over the summed sweep time of the library's phase timing, APD_PHASE_TIMING) beside the RunPatchMatch totals."""
import os, re, subprocess, sys, tempfile, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "apde-mvs_amd"), os.path.join(REPO, "tests")]
import numpy as np
import synth, host_schedule as HS

PARSE = sys.argv[1] == "--parse" if len(sys.argv) > 1 else False  # --parse LOG W H V: summarise an apd log
if PARSE:
    parse_log = sys.argv[2]
    del sys.argv[1:3]
W, H, V = (int(x) for x in sys.argv[1:4]) if len(sys.argv) >= 4 else (3024, 2016, 9)
extra = sys.argv[4:]
apd = os.path.join(REPO, "apde-mvs_amd", "host", "build", "apd")
if PARSE:
    wall, rc, log = float("nan"), 0, parse_log
else:
    sc = synth.make_scene(W, H, V - 1)
    NSRC = int(os.environ.get("TIME_SCAN_NSRC", "10"))
    if NSRC > 0:
        sc.pairs = [pl[:NSRC] for pl in sc.pairs]
    print(f"scene generated ({NSRC or V - 1} sources per view)", flush=True)
    folder = os.environ.get("TIME_SCAN_FOLDER") or tempfile.mkdtemp(prefix="apd_scan_")
    os.makedirs(folder, exist_ok=True)
    HS.write_dense_folder(sc, folder, ext=".png", masks=os.environ.get("TIME_SCAN_SA", "1") == "1")  # TIME_SCAN_SA=0: no sa_masks/ (C3)
    from PIL import Image
    for f in sorted(os.listdir(os.path.join(folder, "images"))):  # re-encode as baseline JPEG
        p = os.path.join(folder, "images", f)
        Image.open(p).save(p[:-4] + ".jpg", quality=95)
        print("jpeg", f, flush=True)
        os.remove(p)
    cmd = [apd, "-d", folder, "--dataset", "ETH3D", "--no_fuse", "true"] + extra
    # the apd stdout goes to a file as it runs (TIME_SCAN_LOG, default under /tmp): a long scan keeps
    # writing, so a watchdog on the output directory sees progress
    log = os.environ.get("TIME_SCAN_LOG", os.path.join(folder, "apd_stdout.log"))
    print(f"scene written ({W}x{H}, {V} views); apd log: {log}", flush=True)
    if os.environ.get("TIME_SCAN_RUN", "1") == "0":  # scene only (the caller runs apd, e.g. under rocprofv3)
        print("command:", " ".join(cmd), flush=True)
        sys.exit(0)
    t0 = time.time()
    with open(log, "w") as lf:
        rc = subprocess.run(cmd, stdout=lf, stderr=subprocess.STDOUT, env=dict(os.environ, APD_PHASE_TIMING="1")).returncode
    wall = time.time() - t0


class _Out:
    stdout = open(log).read()


out = _Out()
if rc != 0:
    print(out.stdout[-3000:])
    sys.exit(rc)
rpm = [int(x) for x in re.findall(r"RunPatchMatch time: (\d+) ms", out.stdout)]
cost = [int(x) for x in re.findall(r"Cost time: (\d+) ms", out.stdout)][:-1]  # the last line is the total
ht = re.findall(r"HostTiming images ([\d.]+) priors ([\d.]+) set\+run ([\d.]+) \(run (\d+)\) results ([\d.]+) epilogue ([\d.]+) emit ([\d.]+)", out.stdout)
if ht:
    a = np.array(ht, float).sum(0) / 1e3
    print("host breakdown (s, summed over problems): images %.2f priors %.2f set+run %.2f (run %.2f, so set %.2f) "
          "results %.2f epilogue %.2f emit %.2f" % (a[0], a[1], a[2], a[3], a[2] - a[3], a[4], a[5], a[6]), flush=True)
print(f"scan {W}x{H} x{V} views: wall {wall:.1f} s, problems {len(rpm)}, RunPatchMatch total {sum(rpm)/1e3:.1f} s, "
      f"per-problem cost total {sum(cost)/1e3:.1f} s, host overhead {wall - sum(rpm)/1e3:.1f} s", flush=True)
# per round / pass: summed RunPatchMatch time and problem count, in log order
cur_round, cur_pass, per, phases = None, None, {}, {}
for line in out.stdout.splitlines():
    m = re.match(r"=+ Round (\d+) =+", line)
    if m:
        cur_round = int(m.group(1))
        continue
    m = re.match(r"=+ iteration (\d+)=+", line)
    if m:
        cur_pass = int(m.group(1))
        continue
    m = re.match(r"RunPatchMatch time: (\d+) ms", line)
    if m:
        k = (cur_round, cur_pass)
        t, n = per.get(k, (0, 0))
        per[k] = (t + int(m.group(1)), n + 1)
        continue
    m = re.match(r"PhaseTiming (\d+) (\d+) iters (\d+) weak (\d+) total ([\d.]+) anchors ([\d.]+) lists ([\d.]+) "
                 r"pairs ([\d.]+) init ([\d.]+) sweep ([\d.]+) post ([\d.]+)", line)
    if m:
        w_, h_, it, wk = (int(m.group(i)) for i in range(1, 5))
        tot, anc, lst, prs, ini, swp, pst = (float(m.group(i)) for i in range(5, 12))
        ph = phases.setdefault((cur_round, cur_pass), dict(px_it=0, weak=0, px=0, total=0.0, anchors=0.0, lists=0.0,
                                                           pairs=0.0, init=0.0, sweep=0.0, post=0.0, iters=it, size=(w_, h_)))
        ph["px_it"] += w_ * h_ * it
        ph["px"] += w_ * h_
        ph["weak"] += wk
        for k_, v_ in (("total", tot), ("anchors", anc), ("lists", lst), ("pairs", prs), ("init", ini), ("sweep", swp), ("post", pst)):
            ph[k_] += v_
for (r, pss), (t, n) in sorted(per.items(), key=lambda kv: (kv[0][0] or 0, kv[0][1] or 0)):
    print(f"round {r} pass {pss}: {n} problems, RunPatchMatch {t / 1e3:.2f} s ({t / max(n, 1):.0f} ms per problem)", flush=True)
    ph = phases.get((r, pss))
    if ph and ph["sweep"] > 0:
        its = max(ph["iters"], 1)
        print(f"    {ph['size'][0]}x{ph['size'][1]}, WEAK {ph['weak'] / max(ph['px'], 1):.3f}: loop body "
              f"{ph['px_it'] / (ph['sweep'] * 1e-3) / 1e6:.1f} Mpix/s per iteration "
              f"({ph['sweep'] / n / its:.1f} ms per iteration), amortised with the pair table "
              f"{ph['px_it'] / ((ph['sweep'] + ph['pairs']) * 1e-3) / 1e6:.1f}; per problem anchors "
              f"{ph['anchors'] / n:.1f} lists {ph['lists'] / n:.1f} pairs {ph['pairs'] / n:.1f} init {ph['init'] / n:.1f} "
              f"sweep {ph['sweep'] / n:.1f} post {ph['post'] / n:.1f} ms", flush=True)
for r in sorted({k[0] for k in per}, key=lambda x: x or 0):
    t = sum(v[0] for k, v in per.items() if k[0] == r)
    print(f"round {r}: RunPatchMatch {t / 1e3:.2f} s", flush=True)
