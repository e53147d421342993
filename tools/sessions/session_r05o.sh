#!/bin/bash
# round 5, session o: K1a sub-regions per XCD (PartArgs::sub_shift) -- the whole
# -m gpu suite, then pool 16 M (489 buckets) with and without them (kernel
# trace + WRITE_SIZE), and the headline against the HEAD library
set -u
R=$(pwd)
OUT=$R/gpurun_out/${1:-r05_o}; mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for mode in sub flat; do
  envs="X=1"; [ $mode = flat ] && envs="NK_NO_XCD_REGIONS=1"
  (cd /tmp && env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr_$mode" -o run \
    -- python3 "$R/bench.py" --pool 16000000 --steps 20 --warmup 5 --inflight 1 --no-cpu-baseline --no-extras \
    > "$OUT/tr_$mode.log" 2>&1) || { tail "$OUT/tr_$mode.log"; exit 1; }
  tail -1 "$OUT/tr_$mode.log" | cut -c1-200
  python3 - "$OUT/tr_$mode/run_kernel_stats.csv" $mode <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if float(r['Percentage']) > 2: print(sys.argv[2], r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
PY
  (cd /tmp && env $envs timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_$mode/pmc1" -o run \
    -- python3 "$R/bench.py" --pool 16000000 --steps 5 --warmup 2 --no-cpu-baseline --no-extras --settle 0 \
    > "$OUT/pmc_$mode.log" 2>&1) || { tail "$OUT/pmc_$mode.log"; exit 1; }
  python3 tools/pmc_summary.py "$OUT/pmc_$mode" "$OUT/pmc_$mode" > /dev/null 2>&1 || true
  python3 -c "import json; d=json.load(open('$OUT/pmc_$mode/pmc_per_kernel_mean.json')); [print('$mode', k[:40], v) for k,v in d.items() if 'k_part' in k or 'hist' in k]"
done
for round in 1 2; do
  for tag in A head; do
    lib=""; [ $tag != A ] && lib=$R/tools/bin/ab/$tag/libneurokmer.so
    NK_AB_LIB=$lib timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $OUT/hl_${tag}_$round.log 2>&1 || { tail $OUT/hl_${tag}_$round.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/hl_${tag}_$round.log').read().strip().splitlines()[-1]); print('$tag', $round, d['ms_per_step'], d['ms_per_step_one_in_flight'], d['roofline']['avg_launch_ms'], d['stage_ms_event_steps'])"
  done
done
