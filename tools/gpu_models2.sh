#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_models.py tests/test_gpu_parity.py -q -p no:cacheprovider > gpurun_out/pt_models.log 2>&1
echo "tests: $(tail -1 gpurun_out/pt_models.log)"; grep FAILED gpurun_out/pt_models.log | head
timeout -k 10 300 python tools/bench_models.py > gpurun_out/models.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/models.log | tail -2
SKGE_RESCAL_VALU=1 timeout -k 10 300 python tools/bench_models.py --models rescal 2>&1 | grep -v amdgpu.ids | tail -1
