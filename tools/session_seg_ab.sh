#!/bin/bash
# neuron-segmented k_xgroup_seg (NK_XG_SEG=1, the default) vs k_xgroup
# (NK_XG_SEG=0): every test that builds a grouped table,
# then interleaved timings of the exact_counts step (tools/exact_ab.py)
set -u
OUT=gpurun_out/${TAG:-seg}
mkdir -p "$OUT"
f="$OUT/pytest_table.log"
timeout -k 10 400 python -u -m pytest tests/test_gpu_table.py tests/test_gpu_parity.py -x -q --timeout 120 \
  --timeout-method thread -k "table or exact or count or kmer_per_neuron or sequence or distinct" \
  > "$f" 2>&1 || { tail -20 "$f"; exit 1; }
tail -1 "$f"
for i in ${ROUNDS:-1 2 3 4}; do
  for v in "NK_XG_SEG=0" "NK_XG_SEG=1"; do
    env $v timeout -k 10 150 python -u tools/exact_ab.py "$v" >> "$OUT/ab.log" 2>&1 || exit $?
  done
done
grep exact_ms "$OUT/ab.log"
