#!/bin/bash
# same-box A/B of the in-tree library against build_abl/$VARIANT on configs 2 / 3 / 4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for r in 1 2; do
  for c in ${CONFIGS:-2 3 4}; do
    for v in cur ${VARIANT:-exact}; do
      if [ $v = cur ]; then lib=""; else lib=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
      SKGE_LIB_PATH=$lib timeout -k 10 300 python bench.py --config $c --no-cpu --steps 20 --warmup 3 > gpurun_out/abc.log 2>&1 || { tail -5 gpurun_out/abc.log; exit 1; }
      python3 -c "
import json; l=[x for x in open('gpurun_out/abc.log') if x.startswith('{')][0]; j=json.loads(l)
lb=j['detail'].get('large_batch') or {}
print('c$c $v', round(j['value']/1e6,2), 'M', j['ms_per_step'], 'ms  nb2', round((lb.get('value') or 0)/1e6,1))"
    done
  done
done
