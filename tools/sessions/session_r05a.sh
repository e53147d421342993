#!/bin/bash
# round 5, session a: pipelined split (K1s beside K1g) -- parity + A/B
set -u
OUT=gpurun_out/${1:-r05_a}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_configs.py::test_uniques_from_kept_records" "tests/test_gpu_configs.py::test_config5_k63_pool256m" \
  > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for i in 1 2 3; do
  for v in 1 0; do
    if [ $v = 1 ]; then export NK_SPLIT_LAUNCHES=1; else unset NK_SPLIT_LAUNCHES; fi
    timeout -k 10 200 python3 -u bench.py --workload config5 --bases 115000000 --steps 20 --warmup 2 \
      --no-side-parity --no-cpu-baseline > $OUT/c5s_g${v}_$i.log 2>&1 || { echo "c5s failed"; tail $OUT/c5s_g${v}_$i.log; exit 1; }
  done
done
unset NK_SPLIT_LAUNCHES
for v in 0 1; do
  if [ $v = 1 ]; then export NK_SPLIT_LAUNCHES=1; else unset NK_SPLIT_LAUNCHES; fi
  timeout -k 10 300 python3 -u bench.py --workload config5 --steps 3 --warmup 1 \
    --no-side-parity --no-cpu-baseline > $OUT/c5_g${v}.log 2>&1 || { echo "c5 failed"; tail $OUT/c5_g${v}.log; exit 1; }
done
for f in $OUT/c5*.log; do
  python3 -c "import json,sys; d=[json.loads(l) for l in open('$f') if l.startswith('{')][-1]; print('$f'.split('/')[-1], d['ms_per_step'], d.get('count_ms_steps'), d['stage_ms_event_steps'])"
done
