#!/bin/bash
# Side measurements of the count paths (not the metric): pools past the
# narrow partition, compat k=63 and --kmer-width=128 at config 2's input size.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/bm_$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc $(tail -1 gpurun_out/bm_$tag.log | python3 -c 'import sys,json
try:
  d=json.loads(sys.stdin.read()); print(d["value"], "Mk/s", d["ms_per_step"], "ms", d["stage_ms"])
except Exception as e: print("no json")')"
  return $rc
}
run p2m && run p16m --pool 16000000 && run p20m --pool 20000000 && \
run c63 --k 63 --pool 2000000 && run w63 --k 63 --kmer-width 128 --pool 2000000 && \
run c63big --k 63 --pool 256000000 && run w63big --k 63 --kmer-width 128 --pool 256000000
