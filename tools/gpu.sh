#!/bin/bash
# One launcher for every GPU-box job (run through gpurun from the repository root):
#
#   gpurun --timeout 900 -- 'bash tools/gpu.sh "tests && bench main --steps 20 && kt c4 -- python3 tools/bench_configs.py c4 1000000"'
#
# The argument is a chain of the steps below joined with && (the chain stops at the first failure, and a
# step that times out, aborts or faults stops it too: nothing more runs on the GPU in that call).  Every
# step runs under its own time limit and writes its log under gpurun_out/.
#
#   tests [pytest args]            -m gpu parity tests (one process)                       -> gpurun_out/tests.log
#   smoke                          __graft_entry__.smoke()                                  -> gpurun_out/smoke.log
#   bench TAG [bench.py args]      python bench.py ...                                      -> gpurun_out/TAG.log
#   py TAG SCRIPT [args]           python SCRIPT args (tools/*.py experiments)               -> gpurun_out/TAG.log
#   kt TAG -- CMD...               rocprofv3 --kernel-trace --stats of CMD                  -> gpurun_out/kt_TAG/
#   pmc TAG "COUNTERS" -- CMD...   one rocprofv3 --pmc pass (its own run; <= the per-block slots,
#                                  MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in separate passes)
#                                                                                           -> gpurun_out/pmc_TAG/
#   sq TAG -- CMD...               the SQ instruction / wait counter pass                    -> gpurun_out/pmc_TAG/
#   lib SO                         later steps load SO instead of hocuspocus_amd/libygm.so (YGM_LIB)
#
# Limits: GPU_STEP_LIMIT (default 300 s) for tests / bench / py, 180 s (SIGKILL) for profiler passes.
set -o pipefail
R=$PWD
mkdir -p "$R/gpurun_out"
LIM=${GPU_STEP_LIMIT:-300}

tests() { timeout -k 10 "$LIM" python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread "$@" > "$R/gpurun_out/tests.log" 2>&1; }
smoke() { timeout -k 10 "$LIM" python -u -c 'import __graft_entry__ as g; g.smoke()' > "$R/gpurun_out/smoke.log" 2>&1; }
bench() { local tag=$1; shift; timeout -k 10 "$LIM" python -u "$R/bench.py" "$@" > "$R/gpurun_out/$tag.log" 2>&1; }
py() { local tag=$1 script=$2; shift 2; timeout -k 10 "$LIM" python -u "$R/$script" "$@" > "$R/gpurun_out/$tag.log" 2>&1; }
lib() { export YGM_LIB=$R/$1; }
_prof() {   # _prof DIR LOG -- profiler args... -- CMD...
  local dir=$1 log=$2; shift 2
  (export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 "$@" > "$log" 2>&1)
}
kt() {
  local tag=$1; shift; [ "$1" = "--" ] && shift
  _prof "$R/gpurun_out/kt_$tag" "$R/gpurun_out/kt_$tag.log" --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_$tag" -o kt -- "$@"
}
pmc() {
  local tag=$1 ctr=$2; shift 2; [ "$1" = "--" ] && shift
  # shellcheck disable=SC2086
  _prof "$R/gpurun_out/pmc_$tag" "$R/gpurun_out/pmc_$tag.log" --pmc $ctr --kernel-trace --output-format csv -d "$R/gpurun_out/pmc_$tag" -o p -- "$@"
}
sq() {
  local tag=$1; shift; [ "$1" = "--" ] && shift
  pmc "$tag" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" -- "$@"
}

[ $# -ge 1 ] || { sed -n 2,24p "$0"; exit 2; }
eval "$1"
