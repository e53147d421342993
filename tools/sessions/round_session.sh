#!/bin/bash
# One end-of-milestone GPU session: the whole -m gpu suite, smoke(), the
# driver's own bench command, and a rocprofv3 kernel trace of a one-in-flight
# bench run; everything under gpurun_out/<tag>/.  Stops at the first failure.
set -u
TAG=${1:-final}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1 || exit $?
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | cut -c1-400
export TMPDIR=/tmp
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 "$R/bench.py" --steps 20 --warmup 5 --inflight 1 --no-cpu-baseline --no-extras \
  > "$OUT/trace.log" 2>&1 || exit $?
echo trace done
