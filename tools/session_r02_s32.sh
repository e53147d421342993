#!/bin/bash
# Round 2, session 32: the final default bench (3 batches in flight on one
# count stream; 50 steps; full CPU baseline + parity + extras), a second
# default run without extras, config 4 at the new default, and smoke.
set -u
mkdir -p gpurun_out/s32
export TMPDIR=/tmp
R=$(pwd)
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); h=d['step_ms_host']; print('$1', d['value'], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), 'steady', round(sorted(h)[len(h)//2],4), d['roofline']['avg_launch_ms'], d['total_spikes'], d.get('inflight_handles_same_results'), (d.get('parity_full') or {}).get('all_equal'))"; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s32/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/s32/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/s32/bench_default.log 2>&1 || { tail -30 gpurun_out/s32/bench_default.log; exit 1; }
summ gpurun_out/s32/bench_default.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras > gpurun_out/s32/bench_default2.log 2>&1 || exit $?
summ gpurun_out/s32/bench_default2.log
timeout -k 10 400 python -u bench.py --workload config4 --steps 20 --no-cpu-baseline > gpurun_out/s32/config4.log 2>&1 || exit $?
summ gpurun_out/s32/config4.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s32/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-extras > $R/gpurun_out/s32/trace.log 2>&1 || exit $?
echo done
