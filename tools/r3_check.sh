#!/bin/bash
# One GPU-box pass (run from the repo root):  bash tools/r3_check.sh <outdir> [bench] [tests] [prof]
# bench: bench.py (default flags) -> bench.json; tests: pytest -m gpu + smoke; prof: rocprofv3 kernel
# stats of the headline bench. Each GPU step has its own time limit. Test failures (exit 1) are
# recorded and the next step still runs; any other failure (time limit, abort, fault) ends the script.
OUT=${1:-gpurun_out/check}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local name=$1 lim=$2; shift 2
  echo "[$(date +%T)] $name" >> "$OUT/steps.log"
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name rc=$rc"; exit $rc; fi
  return 0
}
for what in "$@"; do
  case $what in
    bench) step bench 600 bash -c "python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err" ;;
    tests) step pytest 1100 bash -c "python3 -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1"
           step smoke 300 bash -c "python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1" ;;
    prof) cd /tmp
          step rocprof 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --end-to-end 0 --c2 0 --rich 0 --steps 6 --warmup 1 > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof_bench.err"
          cd "$GRAFT_REPO_ROOT" ;;
  esac
done
echo ok
