#!/bin/bash
# round 5, session f: host FASTQ read costs (CPU only) + the loopback/slice tests
set -u
OUT=gpurun_out/${1:-r05_f}; mkdir -p $OUT
g++ -O2 -std=c++17 -I include -I neurokmer_amd/csrc tools/fqbench.cpp neurokmer_amd/csrc/nk_fqhost.cpp -lpthread -o /tmp/fqbench || exit 1
timeout -k 10 300 /tmp/fqbench /dev/shm/fqbench.fq 16 > $OUT/fqbench16.log 2>&1; rc=$?
cat $OUT/fqbench16.log
[ $rc = 0 ] && timeout -k 10 200 /tmp/fqbench /dev/shm/fqbench.fq 16 16777216 > $OUT/fqbench16_w16.log 2>&1
cat $OUT/fqbench16_w16.log
rm -f /dev/shm/fqbench.fq
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_loopback.py tests/test_gpu_slices.py > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
