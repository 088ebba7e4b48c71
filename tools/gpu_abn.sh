#!/bin/bash
# Same-box A/B of library variants on the default bench, interleaved ROUNDS
# times: cur (the in-tree library) and each of $VARIANTS (build_abl/<v>/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in cur ${VARIANTS:-base}; do
    if [ $v = cur ]; then lib=""; else lib=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
    SKGE_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/abn_$v.log 2>&1 || { tail -5 gpurun_out/abn_$v.log; exit 1; }
    python3 -c "
import json; l=[x for x in open('gpurun_out/abn_$v.log') if x.startswith('{')][0]; j=json.loads(l)
print('$v', round(j['value']/1e6,2), 'M', j['roofline'].get('avg_launch_us'), 'us', round(j['detail'].get('large_batch',{}).get('value',0)/1e6,1), 'M(nb2)', j['ms_per_step'], 'ms/step')"
  done
done
