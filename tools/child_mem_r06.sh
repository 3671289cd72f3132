# Diagnostic children's host memory on the final diag library: the isolated agent at level 1 and level 2 (each child's
# own peak RSS, reported over its pipe), and a level-1 suite with and without the SDMA engines.
set -eo pipefail
O=gpurun_out/childmem
mkdir -p $O
timeout -k 10 60 python tools/child_peak_rss.py --levels 1 | sed 's/^{/{"sdma":"default",/' >> $O/child_peak.jsonl
HSA_ENABLE_SDMA=0 timeout -k 10 60 python tools/child_peak_rss.py --levels 1 | sed 's/^{/{"sdma":"off",/' >> $O/child_peak.jsonl
timeout -k 10 300 python -u tools/agent_soak.py --minutes 2.5 --diag-level 1 --diag-interval 0 --sample 10 --port 19464 --out $O/soak_l1.json > $O/soak_l1.log 2>&1
timeout -k 10 300 python -u tools/agent_soak.py --minutes 2.5 --diag-level 2 --diag-interval 0 --sample 10 --port 19465 --out $O/soak_l2.json > $O/soak_l2.log 2>&1
