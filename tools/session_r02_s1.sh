set -u
mkdir -p gpurun_out/s1
timeout -k 10 120 ./tools/bin/isabench > gpurun_out/s1/isabench.log 2>&1 || exit $?
tail -12 gpurun_out/s1/isabench.log
TAG=abl timeout -k 10 900 bash tools/ablate_k1a.sh run > gpurun_out/s1/ablate.log 2>&1
rc=$?
cat gpurun_out/s1/ablate.log | grep -v "^\s*$" | tail -20
exit $rc
