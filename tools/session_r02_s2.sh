#!/bin/bash
# Round 2, session 2: smoke, the new bench (full CPU baseline + parity, end to
# end, exact_counts step, in-kernel K1a spans), K1a A/B (VGPR uniforms, k >= 16
# mask), the --gpus 2 launch rehearsal and the config-4 workload at N=1.
set -u
mkdir -p gpurun_out/s2
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2/smoke.log 2>&1 || exit $?
tail -2 gpurun_out/s2/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/s2/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/s2/bench_default.log | cut -c1-600
timeout -k 10 600 bash tools/ab_run.sh vuni k16 vk > gpurun_out/s2/ab.log 2>&1 || exit $?
cat gpurun_out/s2/ab.log
timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --no-cpu-baseline > gpurun_out/s2/bench_gpus2.log 2>&1 || exit $?
tail -1 gpurun_out/s2/bench_gpus2.log | cut -c1-400
timeout -k 10 300 python -u bench.py --workload config4 --steps 5 --no-cpu-baseline --no-extras > gpurun_out/s2/bench_c4.log 2>&1 || exit $?
tail -1 gpurun_out/s2/bench_c4.log | cut -c1-400
