# bench.py with and without cpu_pair() pinning, alternated on one box (default steps; no coldstart runs), plus the
# box's CPU topology as this process sees it.
set -eo pipefail
O=gpurun_out/pin
mkdir -p $O
python -c "import os,bench; a=sorted(os.sched_getaffinity(0)); print({'allowed': len(a), 'first': a[:8], 'pair': bench.cpu_pair()})" > $O/topology.txt
for i in 1 2 3; do
  timeout -k 10 150 python bench.py --coldstart-runs 0 > $O/pin_$i.json 2>/dev/null
  timeout -k 10 150 python bench.py --coldstart-runs 0 --no-pin > $O/nopin_$i.json 2>/dev/null
  echo round $i
done
