#!/bin/bash
# round 5, session k: slice segment fused into k_top_final, top-N post into k_slice_adopt -- tests + rehearsal A/B
set -u
OUT=gpurun_out/${1:-r05_k}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_loopback.py tests/test_gpu_slices.py tests/test_gpu_dist.py tests/test_gpu_rccl.py \
  > $OUT/pt_dist.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pt_dist.log; exit 1; }
tail -1 $OUT/pt_dist.log
run() {  # name, env...
  local name=$1; shift
  timeout -k 10 300 env "$@" python3 -u bench.py $BARGS > $OUT/$name.log 2>&1 || { echo "$name failed"; tail $OUT/$name.log; exit 1; }
}
B0="--no-extras --no-cpu-baseline --steps 50"
for i in 1 2 3; do
  BARGS="$B0 --force-dist"; run dist_base_$i NK_AB_LIB=ab_lib/base/libneurokmer.so
  BARGS="$B0 --force-dist"; run dist_new_$i A=1
done
BARGS="$B0"; run plain3 A=1
BARGS="$B0 --inflight 2"; run plain2 A=1
for f in $OUT/dist*.log $OUT/plain*.log; do
  python3 -c "import json,sys; d=[json.loads(l) for l in open('$f') if l.startswith('{')][-1]; print('$f'.split('/')[-1], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), d['inflight'], d['config'].get('finish'), d.get('parity_ranks',{}).get('all_equal') if isinstance(d.get('parity_ranks'),dict) else d.get('parity_ranks'))"
done
