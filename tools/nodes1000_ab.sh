# Why a 1000-node headline (bench.py --nodes 1000) runs slower than the curve's 1000-node row: with and without the
# agent's in-process HIP diagnostics, and the curve row itself, on one box.
set -eo pipefail
O=gpurun_out/n1000
mkdir -p $O
timeout -k 10 150 python bench.py --nodes 1000 --coldstart-runs 0 --curve "" > $O/diag1.json 2> $O/diag1.err
timeout -k 10 150 python bench.py --nodes 1000 --coldstart-runs 0 --curve "" --diag-level 0 > $O/diag0.json 2> $O/diag0.err
timeout -k 10 150 python bench.py --coldstart-runs 0 --curve 1000 > $O/curve.json 2> $O/curve.err
timeout -k 10 150 python bench.py --nodes 1000 --coldstart-runs 0 --curve "" --no-pin > $O/nopin.json 2> $O/nopin.err
