"""Mutation check of the oracle's known-answer tests (CPU only; test infrastructure).

For each mutation below -- one reference rule or quirk of the APD half restated wrongly -- build a
mutated copy of oracle/apd_oracle.c into a temporary liboracle.so and run the known-answer tests
against it (APD_ORACLE_SO). A mutation the tests do not reject ("survived") marks a rule the KATs do
not pin. Usage: python tools/mutate_oracle.py [--json out.json]
"""
import json
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "oracle", "apd_oracle.c")
CFLAGS = "-O2 -mfma -mavx2 -fPIC -fopenmp -ffp-contract=off -fno-fast-math -std=c11 -w".split()

MUTATIONS = [  # (name, reference lines, original text, mutated text)
    ("focal mix 0.25/0.75 -> 0.5/0.5", "APD.cu:586",
     "(float)(0.25 * (double)center_cost + 0.75 * (double)sc)", "(float)(0.5 * (double)center_cost + 0.5 * (double)sc)"),
    ("softmax weights -> plain mean", "APD.cu:431-446",
     "c[i] = o_expf(c[i] - mx); sum += c[i];", "c[i] = 1.0f; sum += c[i];"),
    ("out-of-frame anchor ignores the selected-view bit", "APD.cu:501-507",
     "if (is_set(o->sel[ax + ay * W], s - 1)) { strong_costs[ns++] = COST_MAX;", "if (1) { strong_costs[ns++] = COST_MAX;"),
    ("curve peaks with >=", "APD.cu:2210",
     "if (pc[i - 1] > pc[i] && pc[i + 1] > pc[i]) {\n            is_peak[i] = 1;",
     "if (pc[i - 1] >= pc[i] && pc[i + 1] >= pc[i]) {\n            is_peak[i] = 1;"),
    ("single peak <= 0.15 -> < 0.15", "APD.cu:2226", "(pc[min_peak] <= 0.15f)", "(pc[min_peak] < 0.15f)"),
    ("peak spread / (count - 1) -> / count", "APD.cu:2243", "var /= (float)(count - 1);", "var /= (float)count;"),
    ("peak radius > -> >=", "APD.cu:2220", "abs(min_peak - 30) > weak_peak_radius", "abs(min_peak - 30) >= weak_peak_radius"),
    ("confidence starts at 0", "APD.cu:2303", "int nc = 1;", "int nc = 0;"),
    ("confidence reprojection weight 2 -> 1", "APD.cu:2305,2333",
     "if (sqrtf(dx * dx + dy * dy) <= 2.0f) nc += 2;", "if (sqrtf(dx * dx + dy * dy) <= 2.0f) nc += 1;"),
    ("confidence relative-depth 0.02 -> 0.05", "APD.cu:2336", "fabsf(rd - refd) / rd <= 0.02f", "fabsf(rd - refd) / rd <= 0.05f"),
    ("filter skip threshold removed", "APD.cu:1745", "if (o->cost[c] < 0.001f) return;", "if (o->cost[c] < 0.0f) return;"),
    ("filter even median -> upper middle", "APD.cu:1815-1816", "(n % 2 == 0) ? (f[m - 1] + f[m]) / 2 : f[m]", "f[m]"),
    ("filter y-5 tap condition y > 4 -> y > 5", "APD.cu:1755", "FADD(py > 4, upup - W * 2);", "FADD(py > 5, upup - W * 2);"),
    ("nearest: confidence filter removed", "APD.cu:2463", "if (o->conf[t] < cc) continue;", ""),
    ("nearest: tie -> >=", "APD.cu:2472", "if (o->conf[t] > bc) { bx = tx;", "if (o->conf[t] >= bc) { bx = tx;"),
    ("anchors: >= 6 inliers -> >= 7", "APD.cu:2028", "if (tcnt < 6) continue;", "if (tcnt < 7) continue;"),
    ("anchors: > 3 directions -> > 6", "APD.cu:1965", "if (nsp <= 3) { o->reliable[c] = 0; return; }", "if (nsp <= 6) { o->reliable[c] = 0; return; }"),
    ("anchors: outliers kept", "APD.cu:2064-2067", "{ vx[i] = -1; vy[i] = -1; wgt[i] = FLT_MAX; continue; }", "{ wgt[i] = FLT_MAX; continue; }"),
    ("anchors: cone threshold cos(angle/2) -> cos(angle)", "APD.cu:1900,1939", "if (ca > K.thr) {", "if (ca > K.cos_a) {"),
]

TESTS = ["tests/test_oracle_kat_apd.py", "tests/test_oracle_kat.py"]


def main():
    src = open(SRC).read()
    results = []
    with tempfile.TemporaryDirectory() as td:
        os.symlink(os.path.join(REPO, "include"), os.path.join(td, "include"))  # the source's ../include
        for name, ref, old, new in MUTATIONS:
            n = src.count(old)
            if n == 0:
                results.append({"mutation": name, "ref": ref, "status": "NOT APPLIED (text not found)"})
                continue
            mdir = os.path.join(td, "oracle")
            os.makedirs(mdir, exist_ok=True)
            csrc = os.path.join(mdir, "apd_oracle.c")
            open(csrc, "w").write(src.replace(old, new))
            so = os.path.join(td, "liboracle_mut.so")
            inc = os.path.join(REPO, "include")
            subprocess.run(["gcc", *CFLAGS, "-I", inc, "-shared", "-o", so, csrc,
                            os.path.join(REPO, "oracle", "fusion_oracle.c"), "-lm"], check=True,
                           cwd=os.path.join(REPO, "oracle"))
            env = dict(os.environ, APD_ORACLE_SO=so)
            r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", *TESTS],
                               cwd=REPO, env=env, capture_output=True, text=True)
            killed = r.returncode != 0
            first = next((ln for ln in r.stdout.splitlines() if ln.startswith("FAILED")), "")
            results.append({"mutation": name, "ref": ref, "status": "killed" if killed else "SURVIVED",
                            "by": first.replace("FAILED ", "")[:120]})
            print(f"{'killed  ' if killed else 'SURVIVED'}  {name}  ({ref})  {first[7:90]}", flush=True)
    if "--json" in sys.argv:
        json.dump(results, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
    survived = [r for r in results if r["status"] != "killed"]
    print(f"{len(results) - len(survived)}/{len(results)} mutations killed")
    sys.exit(1 if survived else 0)


if __name__ == "__main__":
    main()
