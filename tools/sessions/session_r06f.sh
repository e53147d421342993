#!/bin/bash
# round 6, session f: world-8 loopback finishes vs the oracle, and bench.py's
# N > 1 path end to end on one GPU (8 loopback ranks, sliced finish, two in flight)
set -u
mkdir -p gpurun_out/r06f
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_loopback.py > gpurun_out/r06f/pytest_loopback.log 2>&1 || { tail -40 gpurun_out/r06f/pytest_loopback.log; exit 1; }
tail -3 gpurun_out/r06f/pytest_loopback.log
timeout -k 10 500 python -u bench.py --loopback 8 --steps 10 --warmup 2 > gpurun_out/r06f/bench_loopback8.log 2> gpurun_out/r06f/bench_loopback8.err || { tail -30 gpurun_out/r06f/bench_loopback8.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r06f/bench_loopback8.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['parallelism'], d.get('parity_ranks',{}).get('all_equal'))"
