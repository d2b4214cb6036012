#!/bin/bash
# Round 4: energy of the Hash feature pass's parts (debug library ablations, timing/energy only) -- tools/power_paths.py
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
NRC_LIB_PATH=neural-radiance-caching_amd/libnrc_amd_debug.so timeout -k 10 300 python tools/power_paths.py --paths f64,hash --hash-knob hash_feat_abl=1,2,4,7,32,36 > gpurun_out/power_hash_abl.json 2> gpurun_out/power_hash_abl.err || { echo "power_paths failed"; tail -20 gpurun_out/power_hash_abl.err; exit 3; }
python -c "
import json; d=json.load(open('gpurun_out/power_hash_abl.json'))
print('idle', d['idle'].get('power_w'))
for p, r in d['paths'].items(): print(p, {k: round(r.get(k),2) for k in ('us_median','power_w','gfx_mhz','nj_per_query')}, 'mJ', round(r['power_w']*r['us_median']*1e-3,1))
"
