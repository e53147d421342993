#!/bin/bash
# Round 3, session 7: lane-tagged wide records, vectorised hit scan and u8 top-N reads
# (hit tiles only): the Gen/Wide/config-5 tests, the config-5 bench + trace.
set -u
mkdir -p gpurun_out/r03_s7
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_boundary.py tests/test_gpu_slices.py tests/test_gpu_rccl.py \
  -k "k1b or kept or config5 or wide or width128 or compat or gen or simulate or batched or kmer_per_neuron or top_rows or forced or sliced or rccl or mixed or file" \
  > gpurun_out/r03_s7/tests.log 2>&1
rc=$?; tail -4 gpurun_out/r03_s7/tests.log; [ $rc -ne 0 ] && exit $rc
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), d['roofline']['avg_launch_ms'])"; }
timeout -k 10 300 python -u bench.py --workload config5 --steps 10 --no-cpu-baseline --no-extras > gpurun_out/r03_s7/c5.log 2>&1 || exit $?
summ gpurun_out/r03_s7/c5.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/r03_s7/prof_c5 -o run -- python3 $ROOT/bench.py --workload config5 --steps 4 --warmup 1 --settle 0 --no-cpu-baseline --no-extras > $ROOT/gpurun_out/r03_s7/prof_c5.log 2>&1 || exit $?
cd $ROOT
f=$(find gpurun_out/r03_s7/prof_c5 -name "*kernel_trace.csv" | head -1)
python3 tools/trace_gaps.py "$f" --steps 1 > gpurun_out/r03_s7/timeline_c5.txt; tail -20 gpurun_out/r03_s7/timeline_c5.txt
