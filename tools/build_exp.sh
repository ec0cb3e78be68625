#!/bin/bash
# Experiment build of libygm.so (tooling): tools/build_exp.sh <name> "<extra hipcc flags>" [source] -> hocuspocus_amd/exp/libygm_<name>.so
# (one kernel file -- ygm_kernels.hip unless named, e.g. ygm_walk.hip -- recompiled with the flags, linked with the
# product's other objects)
set -e
cd "$(dirname "$0")/../hocuspocus_amd/csrc"
make -s -j4 >/dev/null
mkdir -p ../exp build/exp
SRC=${3:-ygm_kernels.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -pthread $2 -c -o build/exp/$1.o $SRC
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -pthread -shared -o ../exp/libygm_$1.so build/exp/$1.o $(ls build/*.o | grep -v -e "/$SRC.o" -e '/diag_')
echo ../exp/libygm_$1.so
