#!/bin/bash
# round 5, session b: config-5 K1g occupancy sensitivity, split launches, kernel trace
set -u
OUT=gpurun_out/${1:-r05_b}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" python3 -u bench.py --workload config5 --steps 3 --warmup 1 \
    --no-side-parity --no-cpu-baseline > $OUT/$name.log 2>&1 || { echo "$name failed"; tail $OUT/$name.log; exit 1; }
}
run g1 NK_SPLIT_LAUNCHES=1
run g1_lds NK_SPLIT_LAUNCHES=1 NK_GEN_DYN_LDS=22000
run g4 NK_SPLIT_LAUNCHES=4
run g16 NK_SPLIT_LAUNCHES=16
run g32 NK_SPLIT_LAUNCHES=32
run g1b NK_SPLIT_LAUNCHES=1
for f in $OUT/g*.log; do
  python3 -c "import json,sys; d=[json.loads(l) for l in open('$f') if l.startswith('{')][-1]; print('$f'.split('/')[-1], d['ms_per_step'], d.get('count_ms_steps'))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/trace -o run -- \
  python3 -u $GRAFT_REPO_ROOT/bench.py --workload config5 --steps 2 --warmup 1 --no-side-parity --no-cpu-baseline \
  > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1 || { echo "trace failed"; tail $GRAFT_REPO_ROOT/$OUT/trace.log; exit 1; }
find $GRAFT_REPO_ROOT/$OUT/trace -name "*kernel_stats.csv" | head -2
