#!/bin/bash
# round 6, session i: K1a's unpadded LDS sort at 512 buckets (three workgroups
# per CU at config 3's pool): the large-pool parity tests, config 3's resident
# count, then its PMC passes and the config-3 side line
set -u
mkdir -p gpurun_out/r06i
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "pools or wide_partition or skewed or ingest_fastq" tests/test_gpu_table.py tests/test_gpu_configs.py::test_config3_fastq_streaming_50mb > gpurun_out/r06i/pytest.log 2>&1 || { tail -40 gpurun_out/r06i/pytest.log; exit 1; }
tail -2 gpurun_out/r06i/pytest.log
timeout -k 10 300 python -u tools/c3_paths.py 31600000 part,18 > gpurun_out/r06i/paths.log 2>&1 || { tail -20 gpurun_out/r06i/paths.log; exit 1; }
cat gpurun_out/r06i/paths.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06i/prof_part -o run --output-format csv -- python3 -u tools/c3_paths.py 31600000 part > gpurun_out/r06i/prof_part.log 2>&1 || exit $?
bash tools/sessions/session_side.sh r06_c3 config3
