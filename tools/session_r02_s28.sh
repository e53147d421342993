#!/bin/bash
# Round 2, session 28: the round's evidence — full GPU suite, smoke, default
# bench (two batches in flight, 50 steps, full CPU baseline + parity +
# extras), a one-at-a-time bench, kernel trace of the default run.
set -u
mkdir -p gpurun_out/s28
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/s28/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s28/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/s28/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s28/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/s28/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/s28/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/s28/bench_default.log | cut -c1-300
timeout -k 10 300 python -u bench.py --inflight 1 --no-cpu-baseline --no-extras > gpurun_out/s28/bench_one_in_flight.log 2>&1 || exit $?
tail -1 gpurun_out/s28/bench_one_in_flight.log | cut -c1-300
timeout -k 10 300 python -u bench.py --inflight 3 --no-cpu-baseline --no-extras > gpurun_out/s28/bench_inflight3.log 2>&1 || exit $?
for f in bench_default bench_one_in_flight bench_inflight3; do python3 -c "import json; d=json.loads(open('gpurun_out/s28/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), d.get('start_host_ms_median_max'))"; done
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s28/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-extras > $R/gpurun_out/s28/trace.log 2>&1 || exit $?
echo done
