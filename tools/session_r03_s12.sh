#!/bin/bash
# Round 3, session 12: the in-library RCCL finish with a gloo process group for
# the host-side coordination (torch's RCCL group measured to slow K1a,
# profiles/r03_s10-s11), interleaved with the plain step and the torch-RCCL form.
set -u
mkdir -p gpurun_out/r03_s12
export TMPDIR=/tmp
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['ms_per_step_one_in_flight'], d['roofline']['avg_launch_ms'], d['config']['collectives'])"; }
B="--steps 30 --warmup 5 --no-cpu-baseline --no-extras"
i=0
for rep in 1 2; do
for v in "plain:--inflight 1" "libgloo:--inflight 1 --force-dist --dist-backend gloo --nk-comm" "libnccl:--inflight 1 --force-dist" "libgloo3:--inflight 3 --force-dist --dist-backend gloo --nk-comm" "plain3:--inflight 3"; do
  name=${v%%:*}_$rep; flags=${v#*:}
  timeout -k 10 200 python -u bench.py $B $flags > gpurun_out/r03_s12/$name.log 2>&1 || exit $?
  summ gpurun_out/r03_s12/$name.log
done
done
