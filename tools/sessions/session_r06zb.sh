#!/bin/bash
# round 6, session zb: the next chunk uploaded from a helper thread while this one is
# parsed and counted: the ingest tests, then the
# 117 MB FASTA file path against the previous build (interleaved)
set -u
O=gpurun_out/r06zb
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "ingest or file or fastq or fasta or gz or config3 or config1 or e2e" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for round in 1 2 3; do
  timeout -k 10 120 python -u tools/fasta_chunks.py 64 >> $O/new.log 2>&1 || exit 1
  NK_AB_LIB=tools/bin/ab/serialup/libneurokmer.so timeout -k 10 120 python -u tools/fasta_chunks.py 64 >> $O/old.log 2>&1 || exit 1
done
grep round $O/new.log; echo old; grep round $O/old.log
R=$(pwd)
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 -u $R/tools/fasta_chunks.py 64 > $R/$O/prof.log 2>&1) || exit $?
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/prof/run_kernel_stats.csv')))[:8]: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1))"
