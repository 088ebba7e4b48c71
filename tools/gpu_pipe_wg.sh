#!/bin/bash
# A/B of the pipelined runner's workgroup size (timing-only variant builds from
# tools/ablate.sh: build_abl/wg512, build_abl/wg1024 vs the default 256)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in ${VARIANTS:-base wg512 wg1024 base}; do
  if [ $v = base ]; then L=""; else L=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
  SKGE_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu > gpurun_out/wg_$v.log 2>&1 || exit $?
  python3 -c "
import json; j=json.loads([l for l in open('gpurun_out/wg_$v.log') if l.startswith('{')][0])
print('$v', j['value'], j['ms_per_step'], j['roofline']['avg_launch_us'], j['detail']['large_batch']['value'])"
done
