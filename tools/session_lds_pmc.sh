#!/bin/bash
# LDS/issue counters per kernel over the bench (one counter set per pass) and
# the VALU operand-form probes of tools/isabench.hip
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/bin/isabench > gpurun_out/isabench.log 2>&1 || exit $?
cat gpurun_out/isabench.log
(cd /tmp && timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1) || exit $?
grep -oE "SQ_(LDS|WAIT|ACTIVE|INSTS_LDS|INST_CYCLES)[A-Z_]*" gpurun_out/counters.txt | sort -u | tr '\n' ' '; echo
bash tools/profile.sh ${TAG:-lds} pmc "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" || exit $?
python3 tools/pmc_summary.py gpurun_out/prof_${TAG:-lds} gpurun_out/pmc_${TAG:-lds} || exit $?
