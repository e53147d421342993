#!/bin/bash
# round 6, session l: config 3 with <= 64 coarse buckets for the pools past
# 4.2 M: parity at the big pools, the resident count, PMC passes, side line
set -u
mkdir -p gpurun_out/r06l
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "pools or wide or skewed" tests/test_gpu_configs.py -k "config3 and not 1gb" > gpurun_out/r06l/pytest.log 2>&1 || { tail -40 gpurun_out/r06l/pytest.log; exit 1; }
tail -2 gpurun_out/r06l/pytest.log
timeout -k 10 300 python -u tools/c3_paths.py 31600000 part,18 > gpurun_out/r06l/paths.log 2>&1 || exit 1
grep mode gpurun_out/r06l/paths.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06l/prof -o run --output-format csv -- python3 -u tools/c3_paths.py 31600000 part > gpurun_out/r06l/prof.log 2>&1 || exit $?
bash tools/sessions/session_side.sh r06_c3 config3
