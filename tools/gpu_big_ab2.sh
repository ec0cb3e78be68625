#!/bin/bash
# Same-box A/B of full-size C3: HEAD build vs this tree with the jump-table variant forced.
mkdir -p gpurun_out && : > gpurun_out/big_ab2.log
c=c3full
for v in head jump compact head2 jump2 compact2; do
  case $v in head*) export YGM_LIB=$PWD/hocuspocus_amd/exp/libygm_head.so; unset YGM_BIG_JUMP_MAX;; jump*) unset YGM_LIB; export YGM_BIG_JUMP_MAX=100000000;; *) unset YGM_LIB; export YGM_BIG_JUMP_MAX=0;; esac
  timeout -k 10 300 python -u bench.py --big $c --no-cpu-baseline --no-yjs > gpurun_out/ab2_${v}.log 2>&1 || exit 1
  echo "$c $v $(tail -1 gpurun_out/ab2_${v}.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d[\"gpu_ms\"],d[\"gpu_runs_ms\"])")" >> gpurun_out/big_ab2.log
done
