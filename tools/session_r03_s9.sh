#!/bin/bash
# Round 3, session 9: the N > 1 step rehearsed on one GPU (1-rank RCCL, the
# in-library finish) against the plain step; a kernel trace of the rehearsal.
set -u
mkdir -p gpurun_out/r03_s9
export TMPDIR=/tmp
ROOT=$(pwd)
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), d.get('collectives'))"; }
B="--steps 20 --warmup 5 --no-cpu-baseline --no-extras"
timeout -k 10 200 python -u bench.py $B --inflight 1 > gpurun_out/r03_s9/plain1.log 2>&1 || exit $?
summ gpurun_out/r03_s9/plain1.log
timeout -k 10 200 python -u bench.py $B --force-dist > gpurun_out/r03_s9/dist1.log 2>&1 || exit $?
summ gpurun_out/r03_s9/dist1.log
timeout -k 10 200 python -u bench.py $B --force-dist --inflight 3 > gpurun_out/r03_s9/dist3.log 2>&1 || exit $?
summ gpurun_out/r03_s9/dist3.log
timeout -k 10 200 python -u bench.py $B --inflight 1 > gpurun_out/r03_s9/plain1b.log 2>&1 || exit $?
summ gpurun_out/r03_s9/plain1b.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/r03_s9/prof_dist -o run -- python3 $ROOT/bench.py --force-dist --steps 6 --warmup 1 --settle 0 --no-cpu-baseline --no-extras > $ROOT/gpurun_out/r03_s9/prof_dist.log 2>&1 || exit $?
cd $ROOT
f=$(find gpurun_out/r03_s9/prof_dist -name "*kernel_trace.csv" | head -1)
python3 tools/trace_gaps.py "$f" --steps 2 > gpurun_out/r03_s9/timeline_dist.txt; tail -40 gpurun_out/r03_s9/timeline_dist.txt
