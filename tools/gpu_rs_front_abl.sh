#!/bin/bash
# RESCAL fused-front role ablations (timing only): config 4 with the in-tree
# library and build_abl/{nodw,nogemm}, kernel stats of each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in cur ${VARIANTS:-nodw nogemm}; do
  if [ $v = cur ]; then lib=""; else lib=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
  SKGE_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/rsabl_$v -o run -- python3 bench.py --config 4 --steps 5 --warmup 1 --no-cpu --large-nb 0 > gpurun_out/rsabl_$v.log 2>&1 || { tail -5 gpurun_out/rsabl_$v.log; exit 1; }
  echo "== $v"; grep -h "k_rescal\|k_apply" $(find gpurun_out/rsabl_$v -name "*kernel_stats.csv") | cut -d, -f1-4
done
