#!/bin/bash
# Round 4: power / clock / energy per query of the product inference paths (tools/power_paths.py)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python tools/power_paths.py > gpurun_out/power_paths.json 2> gpurun_out/power_paths.err || { echo "power_paths failed"; tail -20 gpurun_out/power_paths.err; exit 3; }
cat gpurun_out/power_paths.err
python -c "
import json; d=json.load(open('gpurun_out/power_paths.json'))
print('idle', d['idle'])
for p, r in d['paths'].items(): print(p, {k: r.get(k) for k in ('us_median','power_w','gfx_mhz','nj_per_query','mfma_pipe_share_at_sampled_clock')})
"
