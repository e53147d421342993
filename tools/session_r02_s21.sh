#!/bin/bash
# Round 2, session 21: two batches in flight (bench --inflight 2) vs one,
# plain and in the 1-rank RCCL rehearsal, plus a 2-rank same-GPU gloo launch
# check and a kernel trace of the overlapped plain run.
set -u
mkdir -p gpurun_out/s21
export TMPDIR=/tmp
R=$(pwd)
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), d['roofline']['avg_launch_ms'], 'k1a_ovl', (sum(d.get('k1a_ms_steps_overlapped') or [0])/max(1,len(d.get('k1a_ms_steps_overlapped') or [])) ), 'spikes', d['total_spikes'], d.get('parity_full', {}).get('all_equal'))"; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --steps 20 > gpurun_out/s21/b2.log 2>&1 || { tail -30 gpurun_out/s21/b2.log; exit 1; }
summ gpurun_out/s21/b2.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --steps 20 --inflight 1 > gpurun_out/s21/b1.log 2>&1 || exit $?
summ gpurun_out/s21/b1.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras --steps 40 > gpurun_out/s21/b2_40.log 2>&1 || exit $?
summ gpurun_out/s21/b2_40.log
export MASTER_ADDR=127.0.0.1
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_PORT=29517 timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-extras --force-dist > gpurun_out/s21/d2.log 2>&1 || { tail -30 gpurun_out/s21/d2.log; exit 1; }
summ gpurun_out/s21/d2.log
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_PORT=29518 timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --no-extras --force-dist --inflight 1 > gpurun_out/s21/d1.log 2>&1 || exit $?
summ gpurun_out/s21/d1.log
timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 1 --settle 0 --no-cpu-baseline > gpurun_out/s21/g2.log 2>&1 || { tail -30 gpurun_out/s21/g2.log; exit 1; }
tail -1 gpurun_out/s21/g2.log | cut -c1-200
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s21/trace -o run -- python3 $R/bench.py --steps 6 --warmup 1 --settle 0 --no-cpu-baseline --no-extras > $R/gpurun_out/s21/trace.log 2>&1 || exit $?
echo done
