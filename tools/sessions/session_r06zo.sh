#!/bin/bash
# round 6, session zo: the N > 1 bench path (one-rank RCCL group) with three
# batches in flight, K1a at three or two workgroups per CU (NK_K1A_DYN_LDS)
set -u
O=gpurun_out/r06zo; mkdir -p $O
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --force-dist"
show() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); print('$2', d['ms_per_step'], d['inflight'], d.get('count_stream_device_clock'), d['step_ms_host'][:6])"; }
for round in 1 2; do
  for v in "0:2" "0:3" "10240:3"; do
    dyn=${v%%:*}; inf=${v#*:}
    NK_K1A_DYN_LDS=$dyn timeout -k 10 150 $B --inflight $inf > $O/d${dyn}_i${inf}_$round.log 2>&1 || { tail -20 $O/d${dyn}_i${inf}_$round.log; exit 1; }
    show $O/d${dyn}_i${inf}_$round.log "dyn=$dyn inflight=$inf r$round"
  done
done
