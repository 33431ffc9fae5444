#!/bin/bash
# One GPU-box session of chained steps (run from the repo root): bash tools/gpu_session.sh OUT STEP...
# Steps: parity | tests:<file,file,...> | gputests | smoke | ab:<AB env>:<libA>,<libB>,... | bench[:args] | pmc:<kernel-regex>:<last>:<bench args> | prof[:args]
#        | script:<path>[,args] (bash <path> <step out dir> args)
# Each GPU step has its own time limit; the script stops at the first failure.
set -e
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n+1))
  kind=${step%%:*}; rest=${step#*:}; [ "$rest" = "$step" ] && rest=""
  echo "[$(date +%T)] step $n: $step"
  case $kind in
    parity) timeout -k 10 420 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/s$n.parity.log" 2>&1 ;;
    tests) timeout -k 10 900 python3 -u -m pytest ${rest//,/ } -m gpu -x -v --timeout 500 --timeout-method thread > "$OUT/s$n.tests.log" 2>&1 ;;
    gputests) timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > "$OUT/s$n.gputests.log" 2>&1 ;;
    smoke) timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/s$n.smoke.log" 2>&1 ;;
    ab) env_=${rest%%:*}; libs=${rest#*:}
        env $env_ timeout -k 10 600 python3 -u tools/ab_apd.py ${libs//,/ } > "$OUT/s$n.ab.log" 2>&1 ;;
    bench) timeout -k 10 900 python3 -u bench.py $rest > "$OUT/s$n.bench.json" 2> "$OUT/s$n.bench.err" ;;
    pmc) re=${rest%%:*}; r2=${rest#*:}; last=${r2%%:*}; bargs=${r2#*:}
         bash tools/pmc_c3.sh "$OUT/s$n.pmc" "$re" $bargs > "$OUT/s$n.pmc.log" 2>&1 ;;
    prof) cd /tmp
          timeout -k 10 700 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/s$n.prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --c2 0 --rich 0 --sa 0 --steps 6 --warmup 1 $rest > "$GRAFT_REPO_ROOT/$OUT/s$n.prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/s$n.prof_bench.err"
          cd "$GRAFT_REPO_ROOT" ;;
    script) timeout -k 10 1100 bash ${rest%%,*} "$OUT/s$n.script" ${rest#*,} > "$OUT/s$n.script.log" 2>&1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[$(date +%T)] ok"
