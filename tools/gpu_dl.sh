#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_device_loop.py -q -p no:cacheprovider > gpurun_out/pt_dl.log 2>&1
echo "tests: $(tail -1 gpurun_out/pt_dl.log)"; grep -E "FAILED|Error|assert" gpurun_out/pt_dl.log | head -10
bash tools/gpu_bigbatch.sh
