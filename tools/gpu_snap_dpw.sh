#!/bin/bash
# f-1 kernel: documents-per-wave sweep on the bench's f1 corpus (10k and 100k documents).
mkdir -p gpurun_out
for d in 1 2 4 8 16 64; do
  YGM_SNAP_DPW=$d timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --c2big-docs 0 --c4-docs 0 --no-host-api --no-cpu-baseline --f1-docs 10000 > gpurun_out/dpw_$d.log 2>&1 || exit 1
done
YGM_SNAP_DPW=4 timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --c2big-docs 0 --c4-docs 0 --no-host-api --no-cpu-baseline --f1-docs 100000 > gpurun_out/dpw_4_100k.log 2>&1
