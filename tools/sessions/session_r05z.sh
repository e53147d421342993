#!/bin/bash
# round 5, session z: the headline with 16384-neuron Part buckets (123 buckets,
# K1b 64 KB histograms: two workgroups per CU) against 32768 (62)
set -u
mkdir -p gpurun_out
bash tools/ab_run.sh pbits14
