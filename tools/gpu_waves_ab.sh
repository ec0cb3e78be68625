#!/bin/bash
# Same-box A/B of the large-document tier's workgroup size (YGM_BIG_WAVES) on C5, C3 and full-size C3.
mkdir -p gpurun_out && : > gpurun_out/waves_ab.log
for c in c5 c3 c3full; do
  for v in route2k waves8 waves4 route2k waves8 waves4; do
    YGM_LIB=$PWD/hocuspocus_amd/exp/libygm_$v.so timeout -k 10 300 python -u bench.py --big $c --no-cpu-baseline --no-yjs > gpurun_out/wa_$v.log 2>&1 || exit 1
    echo "$c $v $(tail -1 gpurun_out/wa_$v.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['gpu_ms'],d['gpu_runs_ms'],d['docs_big_tier'],d['docs_seq_tier'],d['parity'][:20])")" >> gpurun_out/waves_ab.log
  done
done
