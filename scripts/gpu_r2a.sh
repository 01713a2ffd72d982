#!/bin/bash
# round-2 first box check: GPU tier, then bench.py at 0/5/20 ms injected shard latency (N=1)
set -o pipefail
out=gpurun_out/r2a
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit $?
for lat in 0 5 20; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --shard-latency-ms $lat > $out/bench_lat$lat.json 2> $out/bench_lat$lat.err || exit $?
  tail -c 400 $out/bench_lat$lat.json
done
