#!/bin/bash
# parity tests, then an A/B of the in-tree library against the given variants
set -u
bash tools/gpu_check.sh || exit $?
bash tools/ab_run.sh "$@"
