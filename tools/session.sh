#!/bin/bash
# r5bi: the c3 line with the statistics on the main stream (--stats-async 0) against asynchronous (the product),
# alternating, product library
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for a in 1 0; do
    timeout -k 10 300 python bench.py --stats-async $a --no-cpu-baseline --no-labelled > gpurun_out/r5bi_${a}_$r.json 2> gpurun_out/r5bi_${a}_$r.err || { tail gpurun_out/r5bi_${a}_$r.err; exit 1; }
    echo -n "async $a: "; python tools/bench_summary.py gpurun_out/r5bi_${a}_$r.json | head -2 | tr '\n' ' '; echo
  done
done
