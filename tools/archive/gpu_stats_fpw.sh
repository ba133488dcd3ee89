#!/bin/bash
# frames per wave of the narrow statistics kernel: c2 and c3 lines at SDRG_STATS_FPW = 1, 2, 4, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for f in 1 2 4; do
    for a in "--config c2" ""; do
      SDRG_STATS_FPW=$f timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-labelled $a > gpurun_out/sfpw.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/sfpw.log; exit 1; }
      tail -1 gpurun_out/sfpw.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); k=d['kernel_ms']; print('fpw $f', '${a:-c3}', d['value'], d['ms_per_step'], k['spectrum_ms'], k['stats_ms'], k['ssb_ms'])"
    done
  done
done
