#!/bin/bash
# prints value / ms_per_step / kernel roofline of every gpurun_out/bench*.log
for f in gpurun_out/bench*.log; do python3 -c "
import json
l=[x for x in open('$f') if x.startswith('{')]
j=json.loads(l[-1]) if l else None
print('$f', j and (j['value'], j['ms_per_step'], j['roofline']['kernel_ms'], j['roofline']['frac']))"; done
