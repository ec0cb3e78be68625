timeout -k 10 120 python -u tools/diag_phases.py > gpurun_out/diag.log 2>&1
