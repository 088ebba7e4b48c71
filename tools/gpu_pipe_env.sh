#!/bin/bash
# TransE bench (default config) under a list of environment settings, same box:
# ENVS="A=1 B=2,C=3 ..." ("-" = none); optional TESTENV: run the device-loop
# tests with that assignment first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
if [ -n "${TESTENV:-}" ]; then
  ( export "$TESTENV"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
      -k "${PYTEST_K:-device_loop or pipe or epoch or runner}" > gpurun_out/pt_env.log 2>&1 ) ; rc=$?
  tail -3 gpurun_out/pt_env.log; [ $rc -ne 0 ] && exit $rc
fi
for v in ${ENVS:--}; do
  ( [ "$v" != "-" ] && for kv in ${v//,/ }; do export "$kv"; done
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu ${BENCH_ARGS:-} > gpurun_out/penv.log 2>&1 ) \
    || { tail -3 gpurun_out/penv.log; exit 1; }
  python -c "
import json; l=[x for x in open('gpurun_out/penv.log') if x.startswith('{')][0]; j=json.loads(l)
print('$v', j['value'], j['ms_per_step'], j['roofline']['avg_launch_us'], j['detail']['large_batch']['value'] if j['detail'].get('large_batch') else None)"
done
