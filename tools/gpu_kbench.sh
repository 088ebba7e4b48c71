#!/bin/bash
# fixed-workload kernel timings (tools/kbench.py) for the current library and variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for cfg in ${CONFIGS:-cur:-:}; do
  name=${cfg%%:*}; rest=${cfg#*:}; v=${rest%%:*}; args=${rest#*:}; args=${args//,/ }
  if [ "$v" = "-" ]; then lib=""; else lib=$PWD/scikit-kge_amd/build_abl/$v/libskgehip.so; fi
  echo -n "$name "
  SKGE_LIB_PATH=$lib timeout -k 10 300 python tools/kbench.py $args 2> gpurun_out/kb_$name.err | tail -1 || exit $?
done
