#!/bin/bash
# Round 2, session 19: kmer_per_neuron by partition (table_kpn) — GPU suite,
# the exact_counts step A/B against the per-key atomic kernel, kernel trace.
set -u
mkdir -p gpurun_out/s19
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/s19/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s19/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/s19/pytest_gpu.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/s19/bench_part.log 2>&1 || exit $?
NK_KPN_ATOMIC=1 timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/s19/bench_atomic.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/s19/bench_part2.log 2>&1 || exit $?
for f in bench_part bench_atomic bench_part2; do python -c "import json,sys; d=json.loads(open('gpurun_out/s19/$f.log').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d.get('exact_counts_step'))"; done
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s19/trace -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/s19/trace.log 2>&1 || exit $?
cd $R && python tools/trace_gaps.py gpurun_out/s19/trace/run_kernel_trace.csv --steps 2 > gpurun_out/s19/timeline.txt 2>&1; grep -E "k_part_keys|k_split|k_kpn|bucket_hist|step" gpurun_out/s19/timeline.txt | tail -12
