#!/bin/bash
# A/B of the persistent grid sizes of the wave / workgroup tiers (resident vs the old fixed 2048 / 512) on the
# full-size C3 batch and the c2_mixed block, in one box.
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --big c3full --no-cpu-baseline > gpurun_out/ab_c3_res.log 2>&1 && \
YGM_WAVE_GRID=2048 YGM_FAST_GRID=512 timeout -k 10 300 python -u bench.py --big c3full --no-cpu-baseline > gpurun_out/ab_c3_old.log 2>&1 && \
timeout -k 10 300 python -u bench.py --big c3full --no-cpu-baseline > gpurun_out/ab_c3_res2.log 2>&1 && \
timeout -k 10 300 python -u bench.py --c2big-docs 0 --c4-docs 0 --f1-docs 0 --no-host-api --no-v2 --no-c3 --no-cpu-baseline > gpurun_out/ab_mx_res.log 2>&1 && \
YGM_WAVE_GRID=2048 YGM_FAST_GRID=512 timeout -k 10 300 python -u bench.py --c2big-docs 0 --c4-docs 0 --f1-docs 0 --no-host-api --no-v2 --no-c3 --no-cpu-baseline > gpurun_out/ab_mx_old.log 2>&1
