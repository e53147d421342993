#!/bin/bash
# round 5, session e: split host files + host FASTQ extraction + fused split
set -u
OUT=gpurun_out/${1:-r05_e}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "ingest or file_streaming or cli_stdout or errors_fail" \
  tests/test_gpu_configs.py -k "config3 or config5_k63 or kept_records or batched_streaming or config1" \
  tests/test_gpu_loopback.py \
  > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
FQ=/dev/shm/nk_r05e.fq
c3() {  # name, env...
  local name=$1; shift
  timeout -k 10 400 env NK_INGEST_PROFILE=1 "$@" python3 -u bench.py --workload config3 --steps 5 --fastq $FQ \
    --no-side-parity --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail $OUT/$name.log; rm -f $FQ; exit 1; }
}
c3 c3_host A=1
c3 c3_dev NK_FASTQ_DEVICE=1
c3 c3_host2 A=1
rm -f $FQ
for f in $OUT/c3*.log; do
  python3 -c "import json,sys; d=[json.loads(l) for l in open('$f') if l.startswith('{')][-1]; print('$f'.split('/')[-1], d['ms_per_step'], d['step_ms_all'], d['end_to_end']['resident_step_ms'])"
  grep "nk ingest" $f | tail -2
done
run() {  # name, env...
  local name=$1; shift
  timeout -k 10 300 env "$@" python3 -u bench.py --workload config5 $BARGS \
    --no-side-parity --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail $OUT/$name.log; exit 1; }
}
BARGS="--steps 3 --warmup 1"
run g1 NK_SPLIT_LAUNCHES=1
run gd A=1
BARGS="--bases 115000000 --steps 20 --warmup 2"
run s_g1 NK_SPLIT_LAUNCHES=1
run s_gd A=1
for f in $OUT/*g*.log; do
  python3 -c "import json,sys; d=[json.loads(l) for l in open('$f') if l.startswith('{')][-1]; c=d.get('count_ms_steps'); print('$f'.split('/')[-1], d['ms_per_step'], sorted(c)[len(c)//2], d['total_spikes'])"
done
