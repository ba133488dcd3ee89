#!/bin/bash
# lab: SSB role maps (SDRG_PIPE_MAP) under the full pipelined c3 step, alternating; one process per run
mkdir -p gpurun_out
for rep in 1 2; do
  for m in ${MAPS:-7B984A653210 7B984A563210 7B986A453210 7B964A853210}; do
    SDRG_PIPE_MAP=$m timeout -k 10 60 python -u tools/lab/step_once.py map_$m >> gpurun_out/map_ab.log 2>&1 || { echo "run $m failed"; tail -5 gpurun_out/map_ab.log; exit 1; }
  done
done
grep "ms/step" gpurun_out/map_ab.log
