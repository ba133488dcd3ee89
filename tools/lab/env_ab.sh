#!/bin/bash
# lab: A/B of per-process env settings under the full pipelined c3 step (tools/lab/step_once.py), alternating.
# usage: ENVS="SDRG_AP_STREAM=0|SDRG_AP_STREAM=1" REPS=3 bash tools/lab/env_ab.sh
mkdir -p gpurun_out
IFS='|' read -ra SETS <<< "${ENVS}"
for rep in $(seq ${REPS:-3}); do
  for e in "${SETS[@]}"; do
    env $e timeout -k 10 60 python -u tools/lab/step_once.py "$e" >> gpurun_out/env_ab.log 2>&1 || { echo "run $e failed"; tail -5 gpurun_out/env_ab.log; exit 1; }
  done
done
grep "ms/step" gpurun_out/env_ab.log | sort
