#!/bin/bash
# alternate the named fftlab binaries (k16 variant, 4096 frames) 3 times: A/B on one box
D=$(dirname "$0")
mkdir -p gpurun_out
for i in 1 2 3; do
  for b in "$@"; do echo "$b: $(timeout -k 5 60 "$D/$b" 4096 k16)" || exit 1; done
done > gpurun_out/ab.log 2>&1
cat gpurun_out/ab.log
