#!/bin/bash
# rocprofv3 kernel trace of tools/kbench.py (per-kernel durations inside the graphs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kbt -o kb -- python3 tools/kbench.py ${KB_ARGS:-} > gpurun_out/kbt.log 2>&1 || exit $?
tail -1 gpurun_out/kbt.log
