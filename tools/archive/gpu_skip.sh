#!/bin/bash
# SSB pipeline role ablation (diagnostic, wrong results): loop cycles with each role's work skipped
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 1; }
timeout -k 10 60 tools/microbench/valu2 || exit 1
for m in ${MASKS:-0x0 0x10 0x60 0x08 0x80 0x70 0xf8}; do
  SDRG_PIPE_SKIP=$m SDRG_PIPE_STAMPS=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --stages ssb > gpurun_out/skip_$m.log 2>&1 || { echo "skip $m failed"; exit 1; }
  echo "skip $m:"; grep "sdrg stamps" gpurun_out/skip_$m.log | head -8 | awk '{print "   ", $4, $5, $7, $10}'
done
