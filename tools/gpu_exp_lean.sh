#!/bin/bash
# lean merge variants (gpurun): every hocuspocus_amd/exp/*.so on C2 100k (EXP_CORPORA), digests vs the product build
mkdir -p gpurun_out
L=gpurun_out/exp_lean.log
: > $L
timeout -k 10 300 python -u tools/exp_lean.py hocuspocus_amd/libygm.so >> $L 2>&1 && \
EXP_CORPORA=${EXP_CORPORA:-c2_100k} timeout -k 10 500 python -u tools/exp_lean.py hocuspocus_amd/exp/*.so >> $L 2>&1
