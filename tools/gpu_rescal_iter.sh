#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_models.py tests/test_gpu_parity.py -q -p no:cacheprovider -k "rescal" > gpurun_out/pt_rs.log 2>&1
echo "tests: $(tail -1 gpurun_out/pt_rs.log)"; grep FAILED gpurun_out/pt_rs.log | head
MODELS=rescal bash tools/gpu_prof_models.sh
grep -v amdgpu gpurun_out/prof_models/log | tail -1
