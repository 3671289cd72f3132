# After the mock apiserver's single-write responses, one box: the driver's bench twice, the sweep mode, and the sweep
# step's breakdown (the earlier numbers on other boxes are the "before": profiles/bench/variants_r06/).
set -eo pipefail
O=gpurun_out/mockfix
mkdir -p $O
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/new_driverargs.json 2> $O/new.err
timeout -k 10 150 python bench.py --mode sweep --coldstart-runs 0 --curve "" --steps 50 --warmup 5 > $O/new_sweep.json 2>> $O/new.err
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/new_driverargs2.json 2>> $O/new.err
timeout -k 10 100 python tools/sweep_breakdown.py > $O/sweep_breakdown.json 2>> $O/new.err
