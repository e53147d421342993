#!/bin/bash
# N = 2 rehearsal on a one-GPU box: bench.py --gpus 2 starts two ranks that
# share the device over gloo; rank 0's line carries parity_ranks (the union of
# both ranks' inputs counted in one call on its GPU vs the 2-rank state)
set -u
OUT=gpurun_out/${TAG:-d2}
mkdir -p "$OUT"
timeout -k 10 600 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_d2.log" 2>&1 || exit $?
tail -1 "$OUT/bench_d2.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["n_gpus"], d["config"]["parallelism"], d["parity_ranks"]["all_equal"], d["parity_ranks"]["total_spikes"], d["parity_ranks"]["sum_currents"])'
