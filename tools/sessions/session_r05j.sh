#!/bin/bash
# round 5, session j: ingest (sync parse, spin pool) tests + window sizes; config 5 with 128 coarse buckets
set -u
OUT=gpurun_out/${1:-r05_j}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "ingest or file_streaming" > $OUT/pt_ingest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pt_ingest.log; exit 1; }
tail -1 $OUT/pt_ingest.log
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py \
  -k "config3 or config5_k63 or kept_records or batched or fused_lif" > $OUT/pt_configs.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pt_configs.log; exit 1; }
tail -1 $OUT/pt_configs.log
FQ=/dev/shm/nk_r05j.fq
c3() {  # name, env...
  local name=$1; shift
  timeout -k 10 400 env NK_INGEST_PROFILE=1 "$@" python3 -u bench.py --workload config3 --steps 10 --fastq $FQ \
    --no-side-parity --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail $OUT/$name.log; rm -f $FQ; exit 1; }
  python3 -c "import json,sys; d=[json.loads(l) for l in open('$OUT/$name.log') if l.startswith('{')][-1]; print('$name', d['ms_per_step'], d['step_ms_all'])"
  grep "nk ingest" $OUT/$name.log | tail -2
}
c3 w64a A=1
c3 w16 NK_FQ_WINDOW=16777216
c3 w32 NK_FQ_WINDOW=33554432
c3 dev NK_FASTQ_DEVICE=1
c3 w64b A=1
rm -f $FQ
timeout -k 10 300 python3 -u bench.py --workload config5 --steps 3 --warmup 1 --no-side-parity --no-cpu-baseline \
  > $OUT/c5.log 2>&1 || { echo "c5 failed"; tail $OUT/c5.log; exit 1; }
python3 -c "import json,sys; d=[json.loads(l) for l in open('$OUT/c5.log') if l.startswith('{')][-1]; c=d.get('count_ms_steps'); print('c5', d['ms_per_step'], sorted(c)[len(c)//2], d['stage_ms_event_steps'], d['total_spikes'])"
