#!/bin/bash
# RESCAL fused front A/B: the RESCAL GPU tests, bench.py --config 4 with the
# fused front off / on / two dW splits (interleaved), kernel stats of the fused run
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -k "${TESTK:-rescal}" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_rf.log 2>&1; rc=$?
tail -3 gpurun_out/t_rf.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for e in ${ENVS:-"SKGE_RESCAL_FUSED=0" "SKGE_RESCAL_FUSED=1" "SKGE_RS_WSTEP_SEP=1"}; do
    env $e timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 3 --no-cpu > gpurun_out/rf.log 2>&1 || { tail -5 gpurun_out/rf.log; exit 1; }
    python3 -c "
import json
j=json.loads([l for l in open('gpurun_out/rf.log') if l.startswith('{')][0])
lb=j['detail'].get('large_batch') or {}
print('$e', round(j['value']/1e6,2), 'M  nb2', round((lb.get('value') or 0)/1e6,2), j['ms_per_step'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/rfprof -o run -- python3 bench.py --config 4 --steps 5 --warmup 1 --no-cpu --large-nb 0 > gpurun_out/rfprof.log 2>&1 || exit $?
grep -h "k_rescal\|k_apply" $(find gpurun_out/rfprof -name "*kernel_stats.csv") | cut -d, -f1-4
