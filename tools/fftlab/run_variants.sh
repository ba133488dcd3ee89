#!/bin/bash
# time fftlab variants (k16 kernel) back to back, twice each to see the spread
D=$(dirname "$0")
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$D"/fftlab_abl0 "$D"/fftlab_abl_*; do
    echo "$(basename $v): $(timeout -k 5 60 $v 4096 k16)"
  done
done > gpurun_out/variants.log 2>&1
cat gpurun_out/variants.log
