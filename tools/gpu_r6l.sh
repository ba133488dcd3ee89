#!/bin/bash
# r6l: issue priority of the DC and AGC waves below the low-pass wave's (lab knob SDRG_PIPE_PRIO, two bits per role):
# product 0x802A00BF (DC, low-pass, AGC at 3, loader at 2), then DC + AGC at 2 / 1 / 0.  In-situ stamps of the SSB stage,
# then the c3 line alternating.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=sdr-for-android-lib_amd/lib
for pm in 0x802A00BF 0x802A00AE 0x802A009D 0x802A008C 0x802A00BF; do
  SDRG_LIB_PATH=$L/libsdrg_lab.so SDRG_PIPE_STAMPS=1 SDRG_PIPE_PRIO=$pm timeout -k 10 200 python tools/lab/step_once.py p_$pm 4 > gpurun_out/r6l_$pm.log 2>&1 || { echo "stamps $pm failed"; tail gpurun_out/r6l_$pm.log; exit 1; }
  echo "prio $pm: $(grep 'wave 1 LPF' gpurun_out/r6l_$pm.log | tail -1 | sed 's/.*steady/steady/') | $(grep ms/step gpurun_out/r6l_$pm.log)"
done
tools/ab.sh -r 2 -o r6l lab lab+p2:SDRG_PIPE_PRIO=0x802A00AE lab+p1:SDRG_PIPE_PRIO=0x802A009D -- python bench.py --steps 200 --warmup 100 --no-cpu-baseline --no-labelled
