#!/bin/bash
# Round 3, session 10: why K1a runs 16 % slower in the 1-rank RCCL rehearsal
# (0.47 vs 0.405 ms, profiles/r03_s9): RCCL present but unused, the Python
# collectives, the in-library finish; plain before and after.
set -u
mkdir -p gpurun_out/r03_s10
export TMPDIR=/tmp
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['stage_ms_event_steps'])"; }
B="--steps 20 --warmup 5 --no-cpu-baseline --no-extras --inflight 1"
for v in plain "init:--force-dist --dist-init-only" "py:--force-dist --dist-python" "lib:--force-dist" "gloo:--force-dist --dist-backend gloo" plain2; do
  name=${v%%:*}; flags=""; [ "$name" != "$v" ] && flags=${v#*:}
  timeout -k 10 200 python -u bench.py $B $flags > gpurun_out/r03_s10/$name.log 2>&1 || exit $?
  summ gpurun_out/r03_s10/$name.log
done
