#!/bin/bash
# same-box A/B of the current library against build_abl/<v> variants on bench.py
# configs (CONFIGS="2 3 4"), each run twice interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for c in ${CONFIGS:-2}; do for rep in 1 2; do for v in cur ${VARIANTS:-old}; do
  if [ $v = cur ]; then lib=""; else lib=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
  SKGE_LIB_PATH=$lib timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu --large-nb 0 > gpurun_out/abc_$v.log 2>&1 || exit $?
  python -c "
import json; l=[x for x in open('gpurun_out/abc_$v.log') if x.startswith('{')][0]; j=json.loads(l)
print('c$c $v', round(j['value']/1e6, 2), j['ms_per_step'], j['roofline'].get('avg_launch_us'))"
done; done; done
