# round-4 probe (tooling): load shapes, the Step2 / snapshot GPU tests, walker whole-line staging A/B with FETCH_SIZE
set -o pipefail
R=$PWD; mkdir -p gpurun_out
(cd tools/proto && for w in 4 8 16; do timeout -k 5 60 ./ldbench 1000000 3328 $w || exit 1; done) > gpurun_out/ldbench.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_step2.py tests/test_snapshot.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_step2.log 2>&1 && \
timeout -k 10 200 python -u tools/exp_c4.py 1000000 hocuspocus_amd/exp/libygm_base.so hocuspocus_amd/exp/libygm_line1.so hocuspocus_amd/exp/libygm_coop.so > gpurun_out/c4ab.log 2>&1 && \
for v in base line1 coop; do
  (export TMPDIR=/tmp YGM_LIB=$R/hocuspocus_amd/exp/libygm_$v.so && timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_f_$v -o p -- python3 tools/exp_c4.py --child 1000000 > $R/gpurun_out/pmc_f_$v.log 2>&1) || exit 1
done
