#!/bin/bash
# A/B of the headline step: a library built from an earlier commit
# (build_ab/<tag>/libneurokmer.so) against the in-tree one, interleaved
set -u
TAG=$1; OUT=gpurun_out/$2; mkdir -p $OUT
for i in 1 2 3 4; do
  order="$TAG new"; [ $((i % 2)) = 0 ] && order="new $TAG"  # alternate which runs first
  for v in $order; do
    lib=""; [ $v != new ] && lib=build_ab/$v/libneurokmer.so
    NK_AB_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras \
      > $OUT/${v}_$i.log 2>&1 || exit $?
  done
done
for f in $OUT/*.log; do
  python3 -c "import json; d=[json.loads(l) for l in open('$f') if l.startswith('{')][-1]; print('$f'.split('/')[-1], d['ms_per_step'], d['ms_per_step_one_in_flight'], d['roofline']['avg_launch_ms'])"
done
