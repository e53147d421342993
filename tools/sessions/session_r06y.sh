#!/bin/bash
# round 6, session y: kernel traces of the 117 MB FASTA file path (device
# parse) for the overlapped ingest (working tree) and the piecewise one (A/B lib)
set -u
O=gpurun_out/r06y
R=$(pwd)
mkdir -p $O
export TMPDIR=/tmp
for v in new old; do
  if [ $v = old ]; then export NK_AB_LIB=$R/tools/bin/ab/previngest/libneurokmer.so; else unset NK_AB_LIB; fi
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/$O/$v -o run -- python3 -u $R/tools/fasta_chunks.py 64 > $R/$O/$v.log 2>&1) || exit $?
  grep round $O/$v.log
done
