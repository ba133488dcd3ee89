#!/bin/bash
# Diagnostic library variant: tools/build_variant.sh NAME "EXTRA_HIPFLAGS" -> sdr-for-android-lib_amd/lib/libsdrg_NAME.so
# (use with SDRG_LIB_PATH=...; never the product library).  Lab builds define SDRG_LAB=1: only they read the lab
# environment knobs (SDRG_PIPE_MAP, SDRG_PIPE_PRIO, SDRG_PIPE_SKIP, SDRG_PIPE_STAMPS, SDRG_CU_SPLIT, ...).
set -e
NAME=$1; FLAGS=$2
D=sdr-for-android-lib_amd; B=$D/build/variant_$NAME; mkdir -p $B
HIP="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -DSDRG_LAB=1 $FLAGS"
CXX="g++ -O2 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -DSDRG_LAB=1"
# SPECTRUM_SRC: an alternative spectrum.hip (A/B of a kernel change in one GPU session)
$HIP -I$D/csrc -Iinclude -c ${SPECTRUM_SRC:-$D/csrc/spectrum.hip} -o $B/spectrum.o
$HIP -c $D/csrc/fftany.hip -o $B/fftany.o
$HIP -I$D/csrc -Iinclude -ffp-contract=off -fno-slp-vectorize -c ${STATS_SRC:-$D/csrc/stats.hip} -o $B/stats.o
$HIP -I$D/csrc -Iinclude -ffp-contract=off -fno-slp-vectorize -c ${SSB_SRC:-$D/csrc/ssb.hip} -o $B/ssb.o
$HIP -ffp-contract=off -c $D/csrc/pulse.hip -o $B/pulse.o
$HIP -c $D/csrc/gather.hip -o $B/gather.o
for f in design engine pulse_bank ingest compat ssb_processor dist; do $CXX -c $D/csrc/$f.cpp -o $B/$f.o; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/lib/libsdrg_$NAME.so $B/spectrum.o $B/fftany.o $B/stats.o \
    $B/ssb.o $B/pulse.o $B/gather.o $B/design.o $B/engine.o $B/pulse_bank.o $B/ingest.o $B/compat.o $B/ssb_processor.o \
    $B/dist.o -lm -lpthread -ldl
echo built $D/lib/libsdrg_$NAME.so
