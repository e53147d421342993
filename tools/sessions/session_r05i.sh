#!/bin/bash
# round 5, session i: config-5 coarse-bucket width A/B, 1-rank multi-GPU rehearsal, config-5 trace
set -u
OUT=gpurun_out/${1:-r05_i}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
run() {  # name, env..., then bench args in BARGS
  local name=$1; shift
  timeout -k 10 300 env "$@" python3 -u bench.py $BARGS > $OUT/$name.log 2>&1 || { echo "$name failed"; tail $OUT/$name.log; exit 1; }
}
BARGS="--workload config5 --steps 3 --warmup 1 --no-side-parity --no-cpu-baseline"
run c5_b20 A=1
run c5_b21 NK_WIDE_BITS=21
run c5_b22 NK_WIDE_BITS=22
run c5_b20b A=1
for f in $OUT/c5_*.log; do
  python3 -c "import json,sys; d=[json.loads(l) for l in open('$f') if l.startswith('{')][-1]; c=d.get('count_ms_steps'); print('$f'.split('/')[-1], d['ms_per_step'], sorted(c)[len(c)//2], d['stage_ms_event_steps'], d['total_spikes'])"
done
B0="--no-extras --no-cpu-baseline --steps 50"
for i in 1 2; do
  BARGS="$B0"; run plain3_$i A=1
  BARGS="$B0 --inflight 2"; run plain2_$i A=1
  BARGS="$B0 --force-dist"; run dist_$i A=1
done
for f in $OUT/plain*.log $OUT/dist*.log; do
  python3 -c "import json,sys; d=[json.loads(l) for l in open('$f') if l.startswith('{')][-1]; print('$f'.split('/')[-1], d['ms_per_step'], d.get('ms_per_step_one_in_flight'), d['inflight'], d['config'].get('finish'))"
done
FQ=/dev/shm/nk_r05i.fq
for i in 1 2 3; do
  timeout -k 10 400 env NK_INGEST_PROFILE=1 python3 -u bench.py --workload config3 --steps 10 --fastq $FQ \
    --no-side-parity --no-cpu-baseline > $OUT/c3_$i.log 2>&1 || { echo "c3 failed"; tail $OUT/c3_$i.log; rm -f $FQ; exit 1; }
  python3 -c "import json,sys; d=[json.loads(l) for l in open('$OUT/c3_$i.log') if l.startswith('{')][-1]; print('c3', d['ms_per_step'], d['step_ms_all'])"
  grep "nk ingest" $OUT/c3_$i.log | tail -3
done
rm -f $FQ
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_c5 -o run -- \
  python3 -u $GRAFT_REPO_ROOT/bench.py --workload config5 --steps 2 --warmup 1 --no-side-parity --no-cpu-baseline \
  > $GRAFT_REPO_ROOT/$OUT/trace_c5.log 2>&1 || { echo "trace failed"; tail $GRAFT_REPO_ROOT/$OUT/trace_c5.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace_dist -o run -- \
  python3 -u $GRAFT_REPO_ROOT/bench.py --force-dist --steps 20 --no-extras --no-cpu-baseline \
  > $GRAFT_REPO_ROOT/$OUT/trace_dist.log 2>&1 || { echo "trace dist failed"; tail $GRAFT_REPO_ROOT/$OUT/trace_dist.log; exit 1; }
echo done
