#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_models.py tests/test_gpu_parity.py -q -p no:cacheprovider -k "hole" > gpurun_out/pt_hole.log 2>&1
echo "tests: $(tail -1 gpurun_out/pt_hole.log)"; grep FAILED gpurun_out/pt_hole.log | head
timeout -k 10 300 python tools/bench_models.py --models hole 2>&1 | grep -v amdgpu | tail -1
