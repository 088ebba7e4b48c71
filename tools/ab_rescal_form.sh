#!/bin/bash
# env-form A/B of the RESCAL front on config 4 (same box)
cd "${GRAFT_REPO_ROOT:-.}"
for f in "" fsplit=2 order=0 order=2 order=4 order=8 fsplit=2,order=4 ""; do
  SKGE_RESCAL_FORM=$f timeout -k 10 200 python bench.py --config 4 --steps 10 --warmup 2 --no-cpu --no-roofline --large-nb 0 > gpurun_out/envab.log 2>&1 || { echo "fail $f"; tail -3 gpurun_out/envab.log; exit 1; }
  python3 -c "
import json,sys;l=[x for x in open('gpurun_out/envab.log') if x.startswith('{')][0];j=json.loads(l);print('form=[$f]',round(j['value']/1e6,2),j['ms_per_step'])"
done
