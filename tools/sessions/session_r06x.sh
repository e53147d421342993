set -u
mkdir -p gpurun_out/r06x
for v in new old; do
  if [ $v = old ]; then export NK_AB_LIB=tools/bin/ab/previngest/libneurokmer.so; else unset NK_AB_LIB; fi
  NK_INGEST_PROFILE=1 timeout -k 10 120 python -u tools/fasta_chunks.py 64 > gpurun_out/r06x/$v.log 2>&1 || exit 1
  echo $v; grep -c "nk ingest" gpurun_out/r06x/$v.log; grep "nk ingest" gpurun_out/r06x/$v.log | tail -4; grep round gpurun_out/r06x/$v.log
done
