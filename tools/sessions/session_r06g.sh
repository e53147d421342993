#!/bin/bash
# round 6, session g: ingest tests (sub-regions in small launches, the
# malformed-record warning), bench.py's torch N > 1 paths after the rank-context
# refactor, and 5 interleaved pairs of the deferred-histogram A/B
set -u
mkdir -p gpurun_out/r06g
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "ingest" > gpurun_out/r06g/pytest_ingest.log 2>&1 || { tail -40 gpurun_out/r06g/pytest_ingest.log; exit 1; }
tail -2 gpurun_out/r06g/pytest_ingest.log
timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 1 --no-parity-ranks > gpurun_out/r06g/bench_gpus2_shared.log 2> gpurun_out/r06g/bench_gpus2_shared.err || { tail -30 gpurun_out/r06g/bench_gpus2_shared.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r06g/bench_gpus2_shared.log').read().strip().splitlines()[-1]); print('gpus2', d['value'], d['ms_per_step'], d['config']['parallelism'])"
timeout -k 10 300 python -u bench.py --force-dist --steps 10 --warmup 1 > gpurun_out/r06g/bench_forcedist.log 2> gpurun_out/r06g/bench_forcedist.err || { tail -30 gpurun_out/r06g/bench_forcedist.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r06g/bench_forcedist.log').read().strip().splitlines()[-1]); print('forcedist', d['value'], d['ms_per_step'], d['config']['collectives'])"
for round in 1 2 3 4 5; do
  for d in off on; do
    log=gpurun_out/r06g/bench_${d}_$round.log
    timeout -k 10 120 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-extras --defer-hist $d > $log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$log').read().strip().splitlines()[-1]); r=d['roofline']; print('$d', $round, d['value'], d['ms_per_step'], d['ms_per_step_one_in_flight'], r['avg_launch_ms'])"
  done
done
