#!/bin/bash
# r5z: the in-launch hand-off's price inside the persistent four-step kernels (1024 x 65536 CS16, spectrum alone):
# per-tile publish (plain + release fence, or write-through sc1 stores) and per-tile acquire, no waiting
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out
D=sdr-for-android-lib_amd/lib
for i in 1 2; do
  for v in base pub1 pub2 acq1 pub1acq; do
    L=$D/libsdrg_$v.so; [ $v == base ] && L=$D/libsdrg.so
    echo "$v: $(SDRG_LIB_PATH=$L timeout -k 10 120 python tools/lab/spec_time.py 65536 cs16 1024 50 2>&1 | tail -1)"
  done
done
cd /tmp
for v in base pub1 pub2 acq1; do
  L=$GRAFT_REPO_ROOT/$D/libsdrg_$v.so; [ $v == base ] && L=$GRAFT_REPO_ROOT/$D/libsdrg.so
  SDRG_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r5z_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/lab/spec_time.py 65536 cs16 1024 50 > $GRAFT_REPO_ROOT/gpurun_out/r5z_$v.log 2>&1 || { echo "prof $v failed"; exit 1; }
done
echo done
