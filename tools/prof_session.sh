#!/bin/bash
# parity tests + bench, then a kernel trace of the bench (rocprofv3)
set -u
bash tools/gpu_check.sh || exit $?
bash tools/profile.sh ${TAG:-s2} trace
