#!/bin/bash
# round 6, session zn: K1a held to two workgroups per CU (extra dynamic LDS,
# NK_K1A_DYN_LDS) so that the finish kernels fit beside it -- the N > 1 bench
# path (one-rank RCCL group, two in flight) and N = 1, interleaved
set -u
O=gpurun_out/r06zn; mkdir -p $O
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras"
show() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', d['ms_per_step'], d.get('count_stream_device_clock'), d['k1a_ms_steps'][:4])"; }
for round in 1 2 3; do
  for v in 0 10240; do
    NK_K1A_DYN_LDS=$v timeout -k 10 150 $B --force-dist > $O/dist_${v}_$round.log 2>&1 || { tail -20 $O/dist_${v}_$round.log; exit 1; }
    show $O/dist_${v}_$round.log "dist dyn=$v r$round"
  done
done
for v in 0 10240; do
  NK_K1A_DYN_LDS=$v timeout -k 10 150 $B > $O/n1_${v}.log 2>&1 || { tail -20 $O/n1_${v}.log; exit 1; }
  show $O/n1_${v}.log "n1 dyn=$v"
done
