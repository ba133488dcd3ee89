#!/bin/bash
# build fftlab variants with k16 ablations (see SDRG_K16_ABLATE in spectrum.hip) and time the k16 kernel
set -e
D=$(dirname "$0")
for m in 0 1 2 3 4 8 16 7 20 31; do
    bash "$D/build.sh" -DSDRG_K16_ABLATE=$m -o "$D/fftlab_abl$m" >/dev/null 2>&1 &
done
wait
ls "$D"/fftlab_abl* >/dev/null
