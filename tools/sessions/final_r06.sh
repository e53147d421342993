#!/bin/bash
# End-of-round session: the whole -m gpu suite, smoke(), the driver's bench
# command, a one-in-flight and a three-in-flight rocprofv3 kernel trace, and the PMC passes over K1a
# that bench.py's roofline.traffic reads (profiles/pmc_count_kernel.json).
set -u
TAG=${1:-r06_final}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
if [ "${NK_FINAL_SKIP_PYTEST:-0}" != 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
fi
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1 || exit $?
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | cut -c1-300
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 "$R/bench.py" --steps 20 --warmup 5 --inflight 1 --no-cpu-baseline --no-extras \
  > "$OUT/trace.log" 2>&1) || exit $?
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace3" -o run \
  -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-extras \
  > "$OUT/trace3.log" 2>&1) || exit $?
echo trace done
B="python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --settle 0"
i=0
for set in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 200 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc/pmc$i" -o run -- $B \
    > "$OUT/pmc$i.log" 2>&1) || exit $?
done
python3 tools/pmc_summary.py "$OUT/pmc" "profiles/$TAG" > "$OUT/pmc_summary.log" 2>&1 || exit $?
cp profiles/pmc_count_kernel.json "profiles/$TAG/pmc_per_kernel_mean.json" "$OUT/"
echo pmc done
