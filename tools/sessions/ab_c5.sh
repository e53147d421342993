#!/bin/bash
# A/B config-5 shape: base library (build_ab/base) vs in-tree
set -u
OUT=gpurun_out/$1; mkdir -p $OUT
for i in 1 2 3; do
  for v in base new; do
    lib=""; [ $v = base ] && lib=build_ab/base/libneurokmer.so
    NK_AB_LIB=$lib timeout -k 10 200 python3 -u bench.py --workload config5 --bases 115000000 --steps 20 --warmup 2 \
      --no-side-parity --no-cpu-baseline > $OUT/c5s_${v}_$i.log 2>&1 || exit $?
  done
done
for v in base new; do
  lib=""; [ $v = base ] && lib=build_ab/base/libneurokmer.so
  NK_AB_LIB=$lib timeout -k 10 300 python3 -u bench.py --workload config5 --steps 3 --warmup 1 \
    --no-side-parity --no-cpu-baseline > $OUT/c5_${v}.log 2>&1 || exit $?
done
for f in $OUT/c5*.log; do
  python3 -c "import json,sys; d=[json.loads(l) for l in open('$f') if l.startswith('{')][-1]; print('$f'.split('/')[-1], d['ms_per_step'], d['stage_ms_event_steps'])"
done
