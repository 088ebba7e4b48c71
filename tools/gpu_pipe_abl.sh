#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in base ${ABL:-noensure noapplye}; do
  if [ $v = base ]; then LIBP=""; else LIBP=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
  SKGE_LIB_PATH=$LIBP timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/b_$v.log 2>&1 || exit $?
  python3 -c "
import json;j=json.loads([l for l in open('gpurun_out/b_$v.log') if l.startswith('{')][0]);print('$v',j['value'],j['ms_per_step'],j['detail']['violations_per_pair'],j['detail']['kernels'])"
done
