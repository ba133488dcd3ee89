#!/bin/bash
# build the spectrum-kernel lab (development harness, not the product)
set -e
D=$(dirname "$0")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I"$D/../../include" -I"$D/../../sdr-for-android-lib_amd/csrc" "$D/fftlab.hip" -o "$D/fftlab" -L"$D/../../sdr-for-android-lib_amd/lib" -lsdrg -Wl,-rpath,'$ORIGIN/../../sdr-for-android-lib_amd/lib' "$@"
