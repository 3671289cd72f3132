# Which device-to-host copy first grows a HIP process by ~180 MiB: one copy per process, pageable and pinned.
set -eo pipefail
O=gpurun_out/copythr
mkdir -p $O
for kib in 4 8 16 32 48 63 64 256; do
  timeout -k 10 60 ./tools/hip_rss_probe.bin x $kib | tail -1 >> $O/pageable.jsonl
  timeout -k 10 60 ./tools/hip_rss_probe.bin x $kib pinned | tail -2 >> $O/pinned.jsonl
done
HSA_ENABLE_SDMA=0 timeout -k 10 60 ./tools/hip_rss_probe.bin x 256 | tail -1 >> $O/nosdma.jsonl
HSA_ENABLE_SDMA=0 timeout -k 10 60 ./tools/hip_rss_probe.bin x 256 pinned | tail -2 >> $O/nosdma.jsonl
