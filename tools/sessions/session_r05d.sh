#!/bin/bash
# round 5, session d: fused hash + split at 6 waves/SIMD -- parity + A/B
set -u
OUT=gpurun_out/${1:-r05_d}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_configs.py::test_uniques_from_kept_records" "tests/test_gpu_configs.py::test_config5_k63_pool256m" \
  > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
run() {  # name, env...
  local name=$1; shift
  timeout -k 10 300 env "$@" python3 -u bench.py --workload config5 $BARGS \
    --no-side-parity --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail $OUT/$name.log; exit 1; }
}
BARGS="--bases 115000000 --steps 20 --warmup 2"
for i in 1 2; do run s_g1_$i NK_SPLIT_LAUNCHES=1; run s_gd_$i A=1; done
BARGS="--steps 3 --warmup 1"
run g1 NK_SPLIT_LAUNCHES=1
run gd A=1
run g16 NK_SPLIT_LAUNCHES=16
for f in $OUT/*g*.log; do
  python3 -c "import json,sys; d=[json.loads(l) for l in open('$f') if l.startswith('{')][-1]; c=d.get('count_ms_steps'); print('$f'.split('/')[-1], d['ms_per_step'], sorted(c)[len(c)//2], d['total_spikes'])"
done
