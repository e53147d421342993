#!/bin/bash
# round 6, session s: no cross-stream wait when a handle's finalize saw its
# readback (quiescent) against the wait every time (NK_ORDER_ALWAYS=1):
# multi-stream tests, interleaved pairs of the driver's command, a trace of each
set -u
O=gpurun_out/r06s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_inflight.py tests/test_gpu_loopback.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for round in 1 2 3 4; do
  for v in new old; do
    if [ $v = old ]; then export NK_ORDER_ALWAYS=1; else unset NK_ORDER_ALWAYS; fi
    log=$O/bench_${v}_$round.log
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('$v', $round, d['value'], d['ms_per_step'], d['ms_per_step_one_in_flight'])"
  done
done
unset NK_ORDER_ALWAYS
R=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace_new -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $R/$O/trace_new.log 2>&1 || exit $?
cd $R
python3 tools/timeline_inflight.py $O/trace_new 20 43 > $O/timeline_new.txt 2>&1; tail -3 $O/timeline_new.txt
