# Host memory of a diagnostic child before / after (a) the v4 epilogue stopped spilling to scratch and (b) the
# host-link test moved to the null stream.  "old" = tools/_old_native (a copy of _native/ whose diag library was built
# by hand from the parent commit's diag.hip), "new" = the in-tree one.  Then the GPU suite on "new".
# (A pinned bounce buffer for host copies was also tried here: no change -- the ~180 MiB comes with the SDMA engines,
# whatever the host memory, tools/copy_threshold.sh.)
set -eo pipefail
O=gpurun_out/scratch2
mkdir -p $O
for i in 1 2; do
  K8SGPU_NATIVE_DIR=tools/_old_native timeout -k 10 120 python tools/child_peak_rss.py --levels 1,2 | sed 's/^{/{"lib":"old",/' >> $O/child_peak.jsonl
  timeout -k 10 120 python tools/child_peak_rss.py --levels 1,2 | sed 's/^{/{"lib":"new",/' >> $O/child_peak.jsonl
done
timeout -k 10 120 python tools/agent_rss.py --first-launch --out $O/first_launch.json > $O/fl.log 2>&1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
