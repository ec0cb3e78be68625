# round-4 probe (tooling): step2 trace, walker A/B (base / whole-line / cooperative staging) with FETCH_SIZE
set -o pipefail
R=$PWD; mkdir -p gpurun_out

timeout -k 10 240 python -u tools/exp_c4.py 1000000 hocuspocus_amd/exp/libygm_base.so hocuspocus_amd/exp/libygm_line1.so hocuspocus_amd/exp/libygm_coop.so > gpurun_out/c4ab.log 2>&1 && \
for v in base coop; do
  (export TMPDIR=/tmp YGM_LIB=$R/hocuspocus_amd/exp/libygm_$v.so && timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_f_$v -o p -- python3 tools/exp_c4.py --child 1000000 > $R/gpurun_out/pmc_f_$v.log 2>&1) || exit 1
done
