#!/bin/bash
# round 6, session j: pools past 4.2 M through the wide count with K1a's rolled
# keys (gen_rolled64): parity, config 3's resident count old/new, PMC passes
set -u
mkdir -p gpurun_out/r06j
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "pools or wide or skewed or ingest_fastq or 16" tests/test_gpu_table.py tests/test_gpu_boundary.py tests/test_gpu_configs.py -k "not 1gb and not 3gbase" > gpurun_out/r06j/pytest.log 2>&1 || { tail -40 gpurun_out/r06j/pytest.log; exit 1; }
tail -2 gpurun_out/r06j/pytest.log
NK_PART_BIG=1 timeout -k 10 300 python -u tools/c3_paths.py 31600000 part > gpurun_out/r06j/paths_partbig.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/c3_paths.py 31600000 part,18,19 > gpurun_out/r06j/paths.log 2>&1 || exit 1
cat gpurun_out/r06j/paths_partbig.log gpurun_out/r06j/paths.log | grep mode
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06j/prof -o run --output-format csv -- python3 -u tools/c3_paths.py 31600000 part > gpurun_out/r06j/prof.log 2>&1 || exit $?
NK_SIDE_ARGS="--no-side-parity" bash tools/sessions/session_side.sh r06_c3w config3
