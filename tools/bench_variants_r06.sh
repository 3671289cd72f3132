# bench.py's other configurations on the final tree, one box: Slack POST per check, sweep mode (re-probe + re-PATCH
# inside the step), and a 1000-node headline.
set -eo pipefail
O=gpurun_out/variants
mkdir -p $O
timeout -k 10 150 python bench.py --slack --coldstart-runs 0 --curve "" > $O/slack.json 2> $O/slack.err
timeout -k 10 150 python bench.py --mode sweep --coldstart-runs 0 --curve "" --steps 50 --warmup 5 > $O/sweep.json 2> $O/sweep.err
timeout -k 10 150 python bench.py --nodes 1000 --coldstart-runs 0 --curve "" > $O/nodes1000.json 2> $O/nodes1000.err
