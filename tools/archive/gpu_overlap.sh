#!/bin/bash
export TMPDIR=/tmp
for cfg in "4096 512" "2048 256" "2048 320" "3072 128" "1024 384"; do
  set -- $cfg
  S_A=$1 SDRG_SPECTRUM_GRID=$2 timeout -k 10 120 python tools/overlap_lab.py 2>&1 | grep S_A || exit 1
done
