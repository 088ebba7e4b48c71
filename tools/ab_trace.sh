#!/bin/bash
# Per-wave traces (tools/pipe_trace.py) of the default build and of
# compile-time variants "name=FLAG" (built on the box by tools/ablate.sh,
# loaded with SKGE_LIB_PATH).  TRACEARGS: pipe_trace.py arguments.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 bash tools/ablate.sh "$@" > gpurun_out/ab_trace_build.log 2>&1 || { tail -5 gpurun_out/ab_trace_build.log; exit 1; }
echo "== base"
timeout -k 10 200 python tools/pipe_trace.py ${TRACEARGS:-} 2>&1 | grep -v amdgpu.ids || exit 1
for v in "$@"; do
  name=${v%%=*}
  echo "== $name"
  SKGE_LIB_PATH=$PWD/scikit-kge_amd/build_abl/$name/libskgehip.so timeout -k 10 200 python tools/pipe_trace.py ${TRACEARGS:-} 2>&1 | grep -v amdgpu.ids || exit 1
done
