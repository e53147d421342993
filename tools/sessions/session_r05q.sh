#!/bin/bash
# round 5, session q: K1a's WRITE_SIZE at pool 16 M without its descriptor
# writes (ablation build nodesc), flat regions and sub-regions per XCD
set -u
R=$(pwd)
OUT=$R/gpurun_out/${1:-r05_q}; mkdir -p $OUT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in "flat::NK_NO_XCD_REGIONS=1" "sub::X=1" "flat_nodesc:$R/tools/bin/ab/nodesc/libneurokmer.so:NK_NO_XCD_REGIONS=1" "sub_nodesc:$R/tools/bin/ab/nodesc/libneurokmer.so:X=1" "hl::X=1:2000000" "hl_nodesc:$R/tools/bin/ab/nodesc/libneurokmer.so:X=1:2000000"; do
  mode=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; rest=${rest#*:}; envs=${rest%%:*}; pool=16000000
  [ "$rest" != "$envs" ] && pool=${rest#*:}
  (cd /tmp && env NK_AB_LIB=$lib $envs timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_$mode/pmc1" -o run \
    -- python3 "$R/bench.py" --pool $pool --steps 5 --warmup 2 --no-cpu-baseline --no-extras --settle 0 \
    > "$OUT/pmc_$mode.log" 2>&1) || { tail "$OUT/pmc_$mode.log"; exit 1; }
  python3 tools/pmc_summary.py "$OUT/pmc_$mode" "$OUT/pmc_$mode" > /dev/null 2>&1 || true
  python3 -c "import json; d=json.load(open('$OUT/pmc_$mode/pmc_per_kernel_mean.json')); [print('$mode', k[:40], round(v['WRITE_SIZE']*1024/1e6,1), 'MB') for k,v in d.items() if 'k_part' in k]"
done
