#!/bin/bash
# Same-box A/B of environment settings on the default bench, interleaved:
#   ENVS="SKGE_LAZY=0 SKGE_LAZY=1" ROUNDS=2 bash tools/gpu_abenv.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for e in ${ENVS}; do
    env $e timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/abenv.log 2>&1 || { tail -5 gpurun_out/abenv.log; exit 1; }
    python3 -c "
import json; l=[x for x in open('gpurun_out/abenv.log') if x.startswith('{')][0]; j=json.loads(l)
print('$e', round(j['value']/1e6,2), 'M', j['roofline'].get('avg_launch_us'), 'us', j['roofline']['achieved'], j['roofline']['unit'], round(j['detail'].get('large_batch',{}).get('value',0)/1e6,1), 'M(nb2)', j['ms_per_step'], 'ms/step')"
  done
done
