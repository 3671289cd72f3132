# Level-1 diagnostic rates with and without the SDMA engines (HSA_ENABLE_SDMA=0, as the agent's isolated level-1
# children run), alternated three times on one box.
set -eo pipefail
O=gpurun_out/sdma_ab
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 120 python -m k8s_gpu_node_checker_amd.ops.diag --level 1 --device 0 --no-p2p --no-rccl --format json > $O/on_$i.json 2>/dev/null
  HSA_ENABLE_SDMA=0 timeout -k 10 120 python -m k8s_gpu_node_checker_amd.ops.diag --level 1 --device 0 --no-p2p --no-rccl --format json > $O/off_$i.json 2>/dev/null
done
