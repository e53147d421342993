#!/bin/bash
# Round 2, session 20: coalesced key extraction (tile_slots) — exact-table GPU
# tests; A/B of the exact_counts step over rocPRIM onesweep configs.
set -u
mkdir -p gpurun_out/s20
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread -k "exact or kmer_per_neuron or table or sequence or adopt or any_n" > gpurun_out/s20/pytest_exact.log 2>&1 || { tail -40 gpurun_out/s20/pytest_exact.log; exit 1; }
tail -2 gpurun_out/s20/pytest_exact.log
for round in 1 2; do
  for tag in A s10i8 s10i12 s8i16 s8i8; do
    lib=""; [ "$tag" != A ] && lib=tools/bin/ab/$tag/libneurokmer.so
    NK_AB_LIB=$lib timeout -k 10 120 python -u tools/exact_ab.py $tag >> gpurun_out/s20/exact_ab.log 2>&1 || { tail -5 gpurun_out/s20/exact_ab.log; exit 1; }
  done
done
grep exact_ms gpurun_out/s20/exact_ab.log
