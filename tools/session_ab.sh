bash tools/gpu_check.sh && bash tools/ab_run.sh prev
