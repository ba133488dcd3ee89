#!/bin/bash
# spectrum16k memory floor: the full kernel (abl 0) vs the same kernel with every FFT step ablated (abl 15:
# convert + |X|^2 + fftshifted stores only), and the bare load / store patterns
D=$(dirname "$0")
mkdir -p gpurun_out
{
for m in 0 15; do echo "abl$m: $(timeout -k 5 60 "$D/fftlab_abl$m" 4096 k16)" || exit 1; done
timeout -k 5 60 "$D/fftlab_abl0" 4096 load-pattern || exit 1
timeout -k 5 60 "$D/fftlab_abl0" 4096 store-pattern || exit 1
} > gpurun_out/floor.log 2>&1
cat gpurun_out/floor.log
