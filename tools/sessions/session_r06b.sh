#!/bin/bash
# round 6, session b: LDS out-of-range test, the fused K1a+K1b tests, and the
# headline with the deferred histogram against without (interleaved)
set -u
mkdir -p gpurun_out/r06b
export TMPDIR=/tmp
timeout -k 5 30 ./tools/bin/oobtest > gpurun_out/r06b/oobtest.log 2>&1 || exit $?
cat gpurun_out/r06b/oobtest.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_inflight.py > gpurun_out/r06b/pytest.log 2>&1 || { tail -40 gpurun_out/r06b/pytest.log; exit 1; }
tail -3 gpurun_out/r06b/pytest.log
for round in 1 2; do
  for d in off on; do
    log=gpurun_out/r06b/bench_${d}_$round.log
    timeout -k 10 120 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extras --defer-hist $d > $log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); r=d['roofline']; print('$d', $round, d['value'], d['ms_per_step'], d['ms_per_step_one_in_flight'], r['avg_launch_ms'], r.get('k1a_alone_ms'))"
  done
done
