#!/bin/bash
# A/B timing on one box: alternates the in-tree library (A) and the variants
# given as tags (tools/bin/ab/<tag>/libneurokmer.so; a tag "env:NAME=VAL" is the
# in-tree library run with that environment variable), bench.py --steps 20,
# two rounds; prints the value, step time and K1's mean launch time per run.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for round in 1 2; do
  for tag in A "$@"; do
    lib=""; envs=""
    case $tag in
      A) ;;
      env:*) envs=${tag#env:} ;;
      *) lib=tools/bin/ab/$tag/libneurokmer.so ;;
    esac
    log=gpurun_out/ab_$(echo "$tag" | tr ':=' '__')_$round.log
    env NK_AB_LIB=$lib $envs timeout -k 10 90 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extras \
      > "$log" 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open('$log').read().strip().splitlines()[-1]); print('$tag', $round, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['avg_launch_ms_events'])"
  done
done
