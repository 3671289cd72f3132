#!/bin/bash
# Round validation on the MI355X box: gpu tests, bench at several cluster sizes, diag level 2, rocprof stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { echo "== $1 ($(date +%T))"; }
step pytest
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
step bench-default
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
for n in 8 1000; do
  step bench-nodes-$n
  timeout -k 10 300 python bench.py --nodes $n --steps $([ $n = 1000 ] && echo 100 || echo 500) --warmup 20 > gpurun_out/bench_nodes$n.json 2> gpurun_out/bench_nodes$n.err || { echo "bench $n failed"; tail -20 gpurun_out/bench_nodes$n.err; exit 1; }
  cat gpurun_out/bench_nodes$n.json
done
step bench-slack
timeout -k 10 300 python bench.py --slack --steps 300 --warmup 20 > gpurun_out/bench_slack.json 2> gpurun_out/bench_slack.err || { echo "bench slack failed"; exit 1; }
cat gpurun_out/bench_slack.json
step diag-level2
timeout -k 10 300 python -m k8s_gpu_node_checker_amd.ops.diag --level 2 > gpurun_out/diag_level2.json 2> gpurun_out/diag_level2.err || { echo "diag failed"; tail -20 gpurun_out/diag_level2.err; cat gpurun_out/diag_level2.json; exit 1; }
cat gpurun_out/diag_level2.json
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_diag -o diag -- python -m k8s_gpu_node_checker_amd.ops.diag --level 2 > gpurun_out/prof_diag.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_diag.log; exit 1; }
find gpurun_out/prof_diag -name "*.csv" | head -20
step agent-soak
timeout -k 10 200 python tools/agent_soak.py --minutes 1 --diag-level 1 --interval 5 --sample 10 --out gpurun_out/agent_soak_round.json > gpurun_out/agent_soak_round.log 2>&1 || { echo "agent soak failed"; tail -20 gpurun_out/agent_soak_round.log; exit 1; }
step contention
timeout -k 10 200 python tools/contention_demo.py --out gpurun_out/contention_round.json > gpurun_out/contention_round.log 2>&1 || { echo "contention demo failed"; tail -20 gpurun_out/contention_round.log; exit 1; }
step node-cycle
timeout -k 10 200 python -m k8s_gpu_node_checker_amd.agent.node_cycle --devices 0 --level 2 --timeout 60 > gpurun_out/node_cycle.json 2> gpurun_out/node_cycle.err || { echo "node cycle failed"; tail -20 gpurun_out/node_cycle.err; exit 1; }
cat gpurun_out/node_cycle.json
step probe-cli
timeout -k 10 60 ./k8s_gpu_node_checker_amd/_native/mi355x-probe --repeat 5 --interval-ms 100 > gpurun_out/probe_cli.jsonl 2>&1 || { echo "probe cli failed"; cat gpurun_out/probe_cli.jsonl; exit 1; }
tail -1 gpurun_out/probe_cli.jsonl
step done
