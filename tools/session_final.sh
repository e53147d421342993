#!/bin/bash
# End-of-round check: the whole -m gpu suite, smoke(), the driver's bench
# command and a one-in-flight kernel trace (tools/round_session.sh), then a
# kernel trace of the exact_counts step (tools/exact_ab.py)
set -u
TAG=${1:-final}
R=$(pwd)
bash tools/round_session.sh "$TAG" || exit $?
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG/xtrace" \
  -o run -- python3 "$R/tools/exact_ab.py" T > "$R/gpurun_out/$TAG/xtrace.log" 2>&1 || exit $?
grep exact_ms "$R/gpurun_out/$TAG/xtrace.log"
