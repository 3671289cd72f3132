# End-of-round evidence on the final tree: the driver's bench invocation (pinned), then the default DaemonSet
# configuration (level 1, process isolation) soaked for 8 minutes with the leak watch.
set -eo pipefail
O=gpurun_out/final_r06
mkdir -p $O
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driverargs.json 2> $O/bench_driverargs.err
timeout -k 10 700 python -u tools/agent_soak.py --minutes 8 --diag-level 1 --diag-interval 0 --sample 10 --out $O/soak_l1_8min.json > $O/soak_l1.log 2>&1
