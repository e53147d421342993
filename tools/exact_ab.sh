#!/bin/bash
# interleaved A/B of the exact_counts step: env settings A and B, N pairs
# usage: tools/exact_ab.sh "<envA>" "<envB>" [pairs]
set -u
A=$1; B=$2; N=${3:-3}
for i in $(seq 1 $N); do
  env $A timeout -k 10 150 python -u tools/exact_ab.py A || exit $?
  env $B timeout -k 10 150 python -u tools/exact_ab.py B || exit $?
done
