#!/bin/bash
# round 5, session l: K1a record stores nontemporal vs plain at pool 16M
# (489 buckets: short segments per tile), kernel trace + WRITE_SIZE each;
# then the end-of-round measurements (tools/sessions/final_r05.sh, no pytest)
set -u
R=$(pwd)
OUT=$R/gpurun_out/${1:-r05_l}; mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for mode in nt plain; do
  (cd /tmp && NK_K1A_STORES=$mode timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_$mode" -o run \
    -- python3 "$R/bench.py" --pool 16000000 --steps 20 --warmup 5 --inflight 1 --no-cpu-baseline --no-extras \
    > "$OUT/tr_$mode.log" 2>&1) || { tail "$OUT/tr_$mode.log"; exit 1; }
  tail -1 "$OUT/tr_$mode.log" | cut -c1-200
  (cd /tmp && NK_K1A_STORES=$mode timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_$mode/pmc1" -o run \
    -- python3 "$R/bench.py" --pool 16000000 --steps 5 --warmup 2 --no-cpu-baseline --no-extras --settle 0 \
    > "$OUT/pmc_$mode.log" 2>&1) || { tail "$OUT/pmc_$mode.log"; exit 1; }
  python3 tools/pmc_summary.py "$OUT/pmc_$mode" "$OUT/pmc_$mode" > /dev/null 2>&1 || true
done
NK_FINAL_SKIP_PYTEST=1 bash tools/sessions/final_r05.sh r05_final
