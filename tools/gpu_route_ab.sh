#!/bin/bash
# Same-box A/B of the wave-tier -> k_merge_big routing threshold (snapshot bytes) on full-size C3 and C3.
mkdir -p gpurun_out && : > gpurun_out/route_ab.log
for c in c3full c3; do
  for v in route2k route1k route512 route2k route1k route512; do
    YGM_LIB=$PWD/hocuspocus_amd/exp/libygm_$v.so timeout -k 10 300 python -u bench.py --big $c --no-cpu-baseline --no-yjs > gpurun_out/ra_$v.log 2>&1 || exit 1
    echo "$c $v $(tail -1 gpurun_out/ra_$v.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['gpu_ms'],d['gpu_runs_ms'],d['docs_big_tier'],d['parity'][:20])")" >> gpurun_out/route_ab.log
  done
done
