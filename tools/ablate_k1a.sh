#!/bin/bash
# K1a (k_part) limiter study.  build: compile the ablation variants here (CPU);
# run: on the GPU box, bench.py --steps 20 for the in-tree library and each
# variant (two rounds), then the PMC passes over the in-tree bench.
#   tools/ablate_k1a.sh build
#   gpurun -- bash tools/ablate_k1a.sh run
set -u
ROOT=$(cd "$(dirname "$0")/.." && pwd)
VARIANTS="nohash:-DNK_ABL_NOHASH norank:-DNK_ABL_NORANK stageonly:-DNK_ABL_STAGEONLY nosort:-DNK_ABL_NOSORT nowrite:-DNK_ABL_NOWRITE"
case ${1:-run} in
  build)
    for v in $VARIANTS; do
      bash "$ROOT/tools/ab_build.sh" "abl_${v%%:*}" "${v#*:}" || exit $?
    done
    ;;
  run)
    cd "$ROOT"
    mkdir -p gpurun_out
    tags=""
    for v in $VARIANTS; do tags="$tags abl_${v%%:*}"; done
    bash tools/ab_run.sh $tags || exit $?
    TAG=${TAG:-abl} bash tools/profile.sh ${TAG:-abl} pmc \
      "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
      "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
      "SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM SQ_BUSY_CU_CYCLES SQ_CYCLES SQ_INST_CYCLES_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" || exit $?
    python3 tools/pmc_summary.py gpurun_out/prof_${TAG:-abl} gpurun_out/pmc_${TAG:-abl} || exit $?
    ;;
esac
