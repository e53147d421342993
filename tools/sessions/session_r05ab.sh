#!/bin/bash
# round 5, session ab: the headline (62 buckets) with the per-XCD sub-regions
# forced (NK_SUB_MIN_BUCKETS=0) against without, interleaved
set -u
mkdir -p gpurun_out
bash tools/ab_run.sh env:NK_SUB_MIN_BUCKETS=0
bash tools/ab_run.sh env:NK_SUB_MIN_BUCKETS=0
