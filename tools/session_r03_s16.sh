#!/bin/bash
# Round 3, session 16: the headline evidence in the driver's own form -- five
# runs of `bench.py --gpus 1 --steps 20 --warmup 5` (medians), a one-in-flight
# rocprofv3 kernel trace with --stats, and the PMC passes for roofline.traffic.
set -u
mkdir -p gpurun_out/r03_s16
export TMPDIR=/tmp
ROOT=$(pwd)
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['ms_per_step_one_in_flight'], d['roofline']['avg_launch_ms'], d['roofline']['valu'].get('frac_of_hash_only'), d.get('parity_full', {}).get('all_equal'))"; }
for i in 1 2 3 4 5; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_s16/bench_$i.log 2>&1 || exit $?
  summ gpurun_out/r03_s16/bench_$i.log
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/r03_s16/trace1 -o run -- python3 $ROOT/bench.py --inflight 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras > $ROOT/gpurun_out/r03_s16/trace1.log 2>&1 || exit $?
cd $ROOT
f=$(find gpurun_out/r03_s16/trace1 -name "*kernel_trace.csv" | head -1)
python3 tools/trace_gaps.py "$f" --steps 3 > gpurun_out/r03_s16/timeline_one_in_flight.txt
tail -12 gpurun_out/r03_s16/timeline_one_in_flight.txt
f=$(find gpurun_out/r03_s16/trace1 -name "*kernel_stats.csv" | head -1); head -12 "$f"
TAG=r03_s16pmc bash tools/profile.sh r03_s16pmc pmc FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES" || exit $?
python3 tools/pmc_summary.py gpurun_out/prof_r03_s16pmc gpurun_out/r03_s16/pmc | tail -14
