#!/bin/bash
# Round 2, session 22: the round's evidence after kmer_per_neuron by partition,
# coalesced key extraction and two batches in flight — full GPU suite, smoke,
# default bench (full CPU baseline + parity + extras), kernel trace.
set -u
mkdir -p gpurun_out/s22
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/s22/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/s22/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/s22/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s22/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/s22/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/s22/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/s22/bench_default.log | cut -c1-400
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s22/trace -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/s22/trace.log 2>&1 || exit $?
echo done
