#!/bin/bash
# r5y: the default bench line with its labelled lines at HEAD (statistics stream created with the engine)
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 400 python bench.py > gpurun_out/r5y_bench$i.json 2> gpurun_out/r5y_bench$i.err || { tail gpurun_out/r5y_bench$i.err; exit 1; }
  python tools/bench_summary.py gpurun_out/r5y_bench$i.json
done
