#!/bin/bash
# Diagnostic library variant: tools/build_variant.sh NAME "EXTRA_HIPFLAGS" -> sdr-for-android-lib_amd/lib/libsdrg_NAME.so
# (use with SDRG_LIB_PATH=...; never the product library)
set -e
NAME=$1; FLAGS=$2
D=sdr-for-android-lib_amd; B=$D/build/variant_$NAME; mkdir -p $B
HIP="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics $FLAGS"
# SPECTRUM_SRC: an alternative spectrum.hip (A/B of a kernel change in one GPU session)
$HIP -I$D/csrc -Iinclude -c ${SPECTRUM_SRC:-$D/csrc/spectrum.hip} -o $B/spectrum.o
$HIP -c $D/csrc/fftany.hip -o $B/fftany.o
$HIP -I$D/csrc -Iinclude -ffp-contract=off -fno-slp-vectorize -c ${STATS_SRC:-$D/csrc/stats.hip} -o $B/stats.o
$HIP -ffp-contract=off -fno-slp-vectorize -c $D/csrc/ssb.hip -o $B/ssb.o
$HIP -ffp-contract=off -c $D/csrc/pulse.hip -o $B/pulse.o
make -s -C $D  # host objects
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/lib/libsdrg_$NAME.so $B/spectrum.o $B/fftany.o $B/stats.o \
    $B/ssb.o $B/pulse.o $D/build/design.o $D/build/engine.o $D/build/pulse_bank.o $D/build/ingest.o $D/build/compat.o \
    $D/build/ssb_processor.o -lm -lpthread
echo built $D/lib/libsdrg_$NAME.so
