#!/bin/bash
# round 6, session k: where config 3's wide count goes: one K1g launch then
# one k_split (NK_SPLIT_LAUNCHES=1) at 2^17 and 2^18 coarse bins
set -u
mkdir -p gpurun_out/r06k
export TMPDIR=/tmp
for m in 17 18; do
  NK_SPLIT_LAUNCHES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06k/prof_s1_$m -o run --output-format csv -- python3 -u tools/c3_paths.py 31600000 $m > gpurun_out/r06k/prof_s1_$m.log 2>&1 || exit $?
  grep mode gpurun_out/r06k/prof_s1_$m.log
  python3 -c "
import csv
for r in list(csv.DictReader(open('gpurun_out/r06k/prof_s1_$m/run_kernel_stats.csv')))[:12]:
    if 'nk::' in r['Name']: print('  ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,1))"
done
