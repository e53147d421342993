#!/bin/bash
# round 6, session t: the handles' ordering events without a system-scope fence
# (default) against fenced (NK_ORDER_FENCE=1), both without the quiescent
# handle's wait; interleaved pairs of the driver's command, traces of both
set -u
O=gpurun_out/r06t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_inflight.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for round in 1 2 3 4; do
  for v in nofence fence; do
    if [ $v = fence ]; then export NK_ORDER_FENCE=1; else unset NK_ORDER_FENCE; fi
    log=$O/bench_${v}_$round.log
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('$v', $round, d['value'], d['ms_per_step'], d['ms_per_step_one_in_flight'])"
  done
done
R=$(pwd)
for v in nofence fence; do
  if [ $v = fence ]; then export NK_ORDER_FENCE=1; else unset NK_ORDER_FENCE; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace_$v -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $R/$O/trace_$v.log 2>&1) || exit $?
  python3 tools/timeline_inflight.py $O/trace_$v 20 43 > $O/timeline_$v.txt 2>&1; tail -1 $O/timeline_$v.txt
done
