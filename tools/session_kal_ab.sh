#!/bin/bash
# K1a<KEYS> segments reserved in 16-record units (NK_KEY_ALIGN16=1, default)
# vs 8 (0): table and parity tests under the default, then interleaved
# timings of the exact_counts step (tools/exact_ab.py)
set -u
OUT=gpurun_out/${TAG:-kal}
mkdir -p "$OUT"
f="$OUT/pytest_table.log"
timeout -k 10 400 python -u -m pytest tests/test_gpu_table.py tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q \
  --timeout 120 --timeout-method thread -k "table or exact or count or kmer_per_neuron or sequence or distinct" \
  > "$f" 2>&1 || { tail -20 "$f"; exit 1; }
tail -1 "$f"
for i in 1 2 3 4; do
  for v in 0 1; do
    NK_KEY_ALIGN16=$v timeout -k 10 150 python -u tools/exact_ab.py "NK_KEY_ALIGN16=$v" >> "$OUT/ab.log" 2>&1 || exit $?
  done
done
grep exact_ms "$OUT/ab.log"
