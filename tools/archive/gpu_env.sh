#!/bin/bash
# time bench stages under environment settings: ENVS="A=1,B=2 C=3" STAGES="all"
export TMPDIR=/tmp
for e in default ${ENVS}; do
  for st in ${STAGES:-all}; do
    if [ $e = default ]; then EV=""; else EV=$(echo $e | tr ',' ' '); fi
    env $EV timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --stages $st > gpurun_out/env_$st.log 2>&1 || { echo "env $e $st failed"; tail -5 gpurun_out/env_$st.log; exit 1; }
    echo "$e $st: $(tail -1 gpurun_out/env_$st.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms"])')"
  done
done
