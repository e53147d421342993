#!/bin/bash
# Side lines of bench.py at their real per-GPU sizes (configs 3-5), each
# preceded by its PMC passes (one counter set per rocprofv3 run) so that the
# line picks up the measured HBM traffic of its count phase.
#   bash tools/sessions/session_side.sh <tag> config5 config4 config3
set -u
TAG=${1:-side}
shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT" "$R/profiles/$TAG"
export TMPDIR=/tmp
for W in "$@"; do
  mkdir -p "$OUT/$W"
  EXTRA=""
  [ "$W" = config4 ] && EXTRA="--shard-of 8"
  if [ "${NK_SIDE_PMC:-1}" = 1 ]; then
    i=0
    for set in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
      i=$((i+1))
      (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$OUT/$W/pmc$i" -o run \
        -- python3 "$R/tools/pmc_side.py" run --workload "$W" > "$OUT/$W/pmc$i.log" 2>&1) || exit $?
    done
    python3 tools/pmc_side.py sum --workload "$W" "$OUT/$W" "profiles/$TAG" > "$OUT/$W/pmc_sum.log" 2>&1 || exit $?
    cp "profiles/pmc_$W.json" "$OUT/" && cp "profiles/$TAG/pmc_${W}_per_kernel.json" "$OUT/" || exit $?
  fi
  timeout -k 10 900 python3 -u bench.py --workload "$W" --steps 5 --warmup 1 $EXTRA ${NK_SIDE_ARGS:-} \
    > "$OUT/bench_$W.log" 2>&1 || exit $?
  tail -1 "$OUT/bench_$W.log" | cut -c1-300
done
