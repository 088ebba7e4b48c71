#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for nb in 18 4 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --nb $nb > gpurun_out/b_nb$nb.log 2>&1 || { tail -3 gpurun_out/b_nb$nb.log; exit 1; }
  python3 -c "
import json;j=json.loads([l for l in open('gpurun_out/b_nb$nb.log') if l.startswith('{')][0]);print('nb=$nb',j['value'],j['ms_per_step'],j['detail']['runner'],j['roofline']['kernel'],j['roofline']['achieved'],j['detail']['kernels'])"
done
