#!/bin/bash
# round 5, session n: the fused gen+split of config 5 -- per-launch times of
# k_gen_split, the same launches with every split deferred (NK_GS_DEFER), a
# workgroup-role interleave (gs_roles), and the launch count
set -u
R=$(pwd)
OUT=$R/gpurun_out/${1:-r05_n}; mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
B="$R/bench.py --workload config5 --steps 3 --warmup 1 --settle 0 --no-side-parity --no-cpu-baseline --no-extras"
run_tr() {  # tag lib envs...
  local tag=$1 lib=$2; shift 2
  (cd /tmp && env NK_AB_LIB=$lib "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
     -d "$OUT/tr_$tag" -o run -- python3 $B > "$OUT/tr_$tag.log" 2>&1) || { tail "$OUT/tr_$tag.log"; exit 1; }
  python3 $R/tools/trace_gs.py "$OUT/tr_$tag" $tag
}
run_tr A "" X=1
run_tr defer "" NK_GS_DEFER=1
run_tr roles $R/tools/bin/ab/gs_roles/libneurokmer.so X=1
for round in 1 2; do
  for v in "A::X=1" "roles:$R/tools/bin/ab/gs_roles/libneurokmer.so:X=1" "L16::NK_SPLIT_LAUNCHES=16" "L64::NK_SPLIT_LAUNCHES=64"; do
    tag=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; envs=${rest#*:}
    env NK_AB_LIB=$lib $envs timeout -k 10 300 python3 $B > "$OUT/pipe_${tag}_$round.log" 2>&1 || { tail "$OUT/pipe_${tag}_$round.log"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/pipe_${tag}_$round.log').read().strip().splitlines()[-1]); print('$tag', $round, d['ms_per_step'], d.get('stage_ms_event_steps'))"
  done
done
