#!/bin/bash
# rocprofv3 evidence for bench.py (one GPU).  Usage: tools/profile.sh <tag> [trace|pmc|list]
# trace: --kernel-trace --stats ; pmc: separate counter passes (never combined
# with trace domains); list: available counters.
set -u
TAG=${1:-r01}
MODE=${2:-trace}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BENCH="python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras"
# counters do not depend on the clock: no settle steps under --pmc
BENCH_PMC="python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --settle 0"
case $MODE in
  list)
    timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1
    ;;
  trace)
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $BENCH > "$OUT/trace.log" 2>&1
    ;;
  pmc)
    shift 2
    i=0
    for set in "$@"; do
      i=$((i+1))
      timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc$i" -o run -- $BENCH_PMC > "$OUT/pmc$i.log" 2>&1 || exit $?
    done
    ;;
esac
