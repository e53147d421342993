#!/bin/bash
# One GPU session: parity tests, then a short bench (+ optional 2-rank rehearsal
# on the single GPU with gloo).  Stops at the first fault / abort / timeout
# (exit codes other than 0 and 1 from pytest).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=20 --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps ${STEPS:-5} --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"
tail -5 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
if [ -n "${DIST2:-}" ]; then
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --bases 30000000 --dist-backend gloo \
    --same-device --no-cpu-baseline > gpurun_out/bench_dist2.log 2>&1
  rc=$?
  echo "dist2 rc=$rc"
  tail -3 gpurun_out/bench_dist2.log
fi
exit $rc
