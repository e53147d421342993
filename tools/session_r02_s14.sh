#!/bin/bash
# Round 2, session 14: two SipHash states side by side (ILP) — in the hash-only
# kernel (dx2) and in K1a (kx2); A/B vs the in-tree library.
set -u
mkdir -p gpurun_out/s14
export TMPDIR=/tmp
timeout -k 10 900 bash tools/ab_run.sh dx2 kx2 > gpurun_out/s14/ab.log 2>&1 || { cat gpurun_out/s14/ab.log; exit 1; }
cat gpurun_out/s14/ab.log
for f in gpurun_out/ab_*_[12].log; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['roofline']['valu'].get('hash_only_ms'))"; done
cp gpurun_out/ab_*_[12].log gpurun_out/s14/
