# The driver's bench invocation and the default one, twice each, on one box.
set -eo pipefail
O=gpurun_out/bfinal
mkdir -p $O
for i in 1 2; do
  timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/driverargs_$i.json 2> $O/driverargs_$i.err
  timeout -k 10 150 python bench.py > $O/default_$i.json 2> $O/default_$i.err
done
