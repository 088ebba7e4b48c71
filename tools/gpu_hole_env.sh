#!/bin/bash
# bench --config 3 under a list of environment settings (same box A/B):
# ENVS="A=1 B=2,C=3 ..." (comma-separated assignments per variant, "-" = none)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for v in ${ENVS:--}; do
  ( [ "$v" != "-" ] && for kv in ${v//,/ }; do export "$kv"; done
    timeout -k 10 300 python bench.py --config ${CONFIG:-3} --steps 20 --warmup 3 --no-cpu --large-nb ${LNB:-0} \
      > gpurun_out/henv.log 2>&1 ) || { tail -3 gpurun_out/henv.log; exit 1; }
  python -c "
import json; l=[x for x in open('gpurun_out/henv.log') if x.startswith('{')][0]; j=json.loads(l)
print('$v', j['value'], j['ms_per_step'])"
done
