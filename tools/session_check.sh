bash tools/gpu_check.sh && bash tools/dist_rehearsal.sh
