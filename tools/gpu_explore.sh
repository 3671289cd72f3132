#!/bin/bash
# GEMM / HBM exploration on one box: the GEMM tests, tools/gemm_explore.py, the HBM lab binary and a rocprofv3 pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu.py -x -q -k "gemm or identity" > gpurun_out/pytest_gemm.log 2>&1 || { echo "gemm tests failed"; tail -30 gpurun_out/pytest_gemm.log; exit 1; }
tail -2 gpurun_out/pytest_gemm.log
timeout -k 10 300 python tools/gemm_explore.py > gpurun_out/gemm_explore.log 2>&1 || { echo "gemm explore failed"; tail -20 gpurun_out/gemm_explore.log; exit 1; }
cat gpurun_out/gemm_explore.log
timeout -k 10 120 ./tools/hbm_explore.bin 4096 > gpurun_out/hbm_explore.log 2>&1 || { echo "hbm explore failed"; tail gpurun_out/hbm_explore.log; exit 1; }
cat gpurun_out/hbm_explore.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gemm -o run -- python tools/gemm_explore.py > gpurun_out/prof_gemm.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_gemm.log; exit 1; }
find gpurun_out/prof_gemm -name "*stats*" | head
