# RCCL / fabric GPU tests, then the mi355x-fabric CLI over 1M-1G messages.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 180 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "rccl or fabric" > gpurun_out/pytest_fabric.log 2>&1 || { echo "fabric tests failed"; tail -40 gpurun_out/pytest_fabric.log; exit 1; }
tail -4 gpurun_out/pytest_fabric.log
NCCL_DEBUG=WARN timeout -k 10 180 python -m k8s_gpu_node_checker_amd.ops.fabric --sizes 1M,64M,256M,1G > gpurun_out/fabric_cli.json 2> gpurun_out/fabric_cli.err || { echo "fabric cli failed"; tail -20 gpurun_out/fabric_cli.err; cat gpurun_out/fabric_cli.json; exit 1; }
cat gpurun_out/fabric_cli.json
