#!/bin/bash
# Device ISA of the product kernels (gfx950), one normalised .s per translation unit, for "this cleanup changes no
# instruction" checks:  tools/isa/dump.sh OUTDIR   then   diff -r OUTDIR_before OUTDIR_after
# (the same flags as sdr-for-android-lib_amd/Makefile; comments, debug-line and file directives dropped)
set -e
OUT=${1:?outdir}
mkdir -p $OUT
S=sdr-for-android-lib_amd/csrc
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics --offload-device-only -S -I include -I $S"
for u in spectrum fftany stats ssb pulse gather; do
  extra=""
  case $u in stats|ssb|pulse) extra="-ffp-contract=off" ;; esac
  case $u in stats|ssb) extra="$extra -fno-slp-vectorize" ;; esac
  /opt/rocm/bin/hipcc $F $extra $S/$u.hip -o $OUT/$u.raw.s 2>/dev/null
  grep -vE '^\s*(;|\.file|\.loc|\.ident|\.section\s+\.debug|\.amdgpu_metadata)' $OUT/$u.raw.s | sed -e 's/\s*;.*$//' -e 's/__hip_cuid_[0-9a-f]*/__hip_cuid/g' > $OUT/$u.s
  rm $OUT/$u.raw.s
done
