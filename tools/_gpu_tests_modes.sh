#!/bin/bash
# GPU parity suite in the default snappy mode and with page mode forced (bitmap discovery)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/gpu_all.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/gpu_all.log; exit 1; }
tail -1 gpurun_out/gpu_all.log
DK_SNAPPY_MODE=page timeout -k 10 500 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/gpu_page.log 2>&1 || { echo pytest page failed; tail -30 gpurun_out/gpu_page.log; exit 1; }
tail -1 gpurun_out/gpu_page.log
