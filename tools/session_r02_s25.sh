#!/bin/bash
# Round 2, session 25: the multi-rank step with two batches in flight, the next
# count enqueued once the all-reduce is (dist.finalize_step between=), in the
# 1-rank RCCL rehearsal (two rounds), plus the dist GPU tests and a 2-rank
# same-GPU gloo launch check.
set -u
mkdir -p gpurun_out/s25
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1
R=$(pwd)
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); h=d['step_ms_host']; print('$1', d['value'], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), 'steady', round(sorted(h)[len(h)//2],4), d['total_spikes'], d.get('inflight_handles_same_results'))"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_slices.py tests/test_gpu_inflight.py -x -q --timeout 300 --timeout-method thread > gpurun_out/s25/pytest.log 2>&1 || { tail -30 gpurun_out/s25/pytest.log; exit 1; }
tail -1 gpurun_out/s25/pytest.log
port=29600
for round in 1 2; do
  for m in 1 2; do
    port=$((port+1))
    WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_PORT=$port timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --force-dist --inflight $m > gpurun_out/s25/d${m}_$round.log 2>&1 || { tail -30 gpurun_out/s25/d${m}_$round.log; exit 1; }
    summ gpurun_out/s25/d${m}_$round.log
  done
done
timeout -k 10 300 python -u bench.py --gpus 2 --steps 6 --warmup 1 --settle 0 --no-cpu-baseline --inflight 2 > gpurun_out/s25/g2.log 2>&1 || { tail -30 gpurun_out/s25/g2.log; exit 1; }
tail -1 gpurun_out/s25/g2.log | cut -c1-240
cd /tmp && WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_PORT=29699 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s25/trace -o run -- python3 $R/bench.py --steps 12 --warmup 1 --settle 0.1 --no-cpu-baseline --no-extras --force-dist --inflight 2 > $R/gpurun_out/s25/trace.log 2>&1 || exit $?
echo done
