#!/bin/bash
# Round 3, session 1: simulate_spikes_auto, sharded-state refusals, rows past
# top_n by threshold + select, 1-rank RCCL (torch and in-library comm), the
# bounded batched count (incl. > 2^32 positions); benches: plain, and the
# 1-rank RCCL rehearsal through the library communicator vs from Python.
set -u
mkdir -p gpurun_out/r03_s1
export TMPDIR=/tmp
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), d['roofline']['avg_launch_ms'], d['config'].get('collectives'))"; }
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --force-dist --no-cpu-baseline --no-extras > gpurun_out/r03_s1/reh_comm_$r.log 2>&1 || exit $?
  summ gpurun_out/r03_s1/reh_comm_$r.log
  timeout -k 10 300 python -u bench.py --force-dist --dist-python --no-cpu-baseline --no-extras > gpurun_out/r03_s1/reh_py_$r.log 2>&1 || exit $?
  summ gpurun_out/r03_s1/reh_py_$r.log
done
timeout -k 10 600 python -u bench.py --gpus 2 --steps 10 --no-cpu-baseline --no-extras > gpurun_out/r03_s1/gloo2.log 2>&1 || exit $?
tail -c 1200 gpurun_out/r03_s1/gloo2.log
