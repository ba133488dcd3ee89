#!/bin/bash
# r6n: per-role stamps of the configs[2] variant (NCO + 127 taps) against the reference chain, SSB stage alone and all
# stages (lab build "lab").
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
for nco in 0 1; do
  for st in 4 31; do
    LAB_NCO=$nco SDRG_LIB_PATH=$L/libsdrg_lab.so SDRG_PIPE_STAMPS=1 timeout -k 10 200 python tools/lab/step_once.py nco${nco}_$st $st > gpurun_out/r6n_nco${nco}_$st.log 2>&1 || { echo "stamps nco$nco/$st failed"; tail gpurun_out/r6n_nco${nco}_$st.log; exit 1; }
    echo "== nco $nco stages $st"; grep -v "abs entry" gpurun_out/r6n_nco${nco}_$st.log | grep -E "wave|ms/step" | sed 's/last:.*steady/steady/' | tail -13
  done
done
