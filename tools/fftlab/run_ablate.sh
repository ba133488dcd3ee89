#!/bin/bash
D=$(dirname "$0")
mkdir -p gpurun_out
for m in 0 1 2 3 4 8 16 7 20 31; do
    echo "ablate $m: $(timeout -k 5 60 "$D/fftlab_abl$m" 4096 k16)"
done > gpurun_out/ablate.log 2>&1
timeout -k 5 60 "$D/fftlab_abl0" 4096 load-pattern >> gpurun_out/ablate.log 2>&1
timeout -k 5 60 "$D/fftlab_abl0" 4096 store-pattern >> gpurun_out/ablate.log 2>&1
cat gpurun_out/ablate.log
