#!/bin/bash
# owner-apply runner timing ablations (build_abl/{noa,allsole}, NOT correct builds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in cur ${VARIANTS:-noa allsole}; do
  if [ $v = cur ]; then lib=""; else lib=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
  for own in 0 1; do
    SKGE_PIPE_OWNER=$own SKGE_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 2 --large-nb 0 > gpurun_out/oabl.log 2>&1 || { tail -5 gpurun_out/oabl.log; exit 1; }
    python3 -c "
import json; l=[x for x in open('gpurun_out/oabl.log') if x.startswith('{')][0]; j=json.loads(l)
print('$v own=$own', round(j['value']/1e6,2), 'M', j['roofline'].get('avg_launch_us'), 'us')"
  done
done
