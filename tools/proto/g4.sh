set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/proto/big_probe.py diagds > gpurun_out/big_probe_ds.log 2>&1
export BIG_MB=10
bash tools/gpu.sh "sq big10 -- python3 tools/proto/big_probe.py"
