#!/bin/bash
# Round 2, session 12: file-ingest buffers kept by the handle — ingest parity
# tests and the bench's end-to-end figures.
set -u
mkdir -p gpurun_out/s12
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_boundary.py -m gpu -x -q -k "ingest or file or fastq or fasta or stream or config3 or golden or cli" --timeout 600 --timeout-method thread > gpurun_out/s12/pytest.log 2>&1 || { tail -40 gpurun_out/s12/pytest.log; exit 1; }
tail -2 gpurun_out/s12/pytest.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/s12/bench.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/s12/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], json.dumps(d['end_to_end']), json.dumps(d['exact_counts_step']))"
