#!/bin/bash
# Box A/B in alternation of the fake apiservers' GC policy: A = NCC_FAKEAPI_GC=collect (gen-1 collection +
# freeze every 5 s), B = freeze every second without collecting.  Driver shape at 0 ms, then 5 ms shard RTT;
# a last pair with the loop-lag monitor on (stall log per arm).
set -o pipefail
out=${1:-gpurun_out/ab_fakegc}
pairs=${2:-3}
mkdir -p "$out"
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 300 env "$@" > $out/$name.json 2> $out/$name.err || exit $?
  python scripts/box/summarize.py $out/$name.json
}
for lat in 0 5; do
  for i in $(seq 1 $pairs); do
    run prev_l${lat}_$i NCC_FAKEAPI_GC=collect python bench.py --steps 20 --warmup 5 --shard-latency-ms $lat
    run cur_l${lat}_$i NCC_FAKEAPI_GC=freeze python bench.py --steps 20 --warmup 5 --shard-latency-ms $lat
  done
done
run prev_lag NCC_FAKEAPI_GC=collect NCC_LOOP_LAG_MS=10 NCC_LOOP_LAG_FILE=$PWD/$out/prev_lag.jsonl python bench.py --steps 20 --warmup 5 --shard-latency-ms 5
run cur_lag NCC_FAKEAPI_GC=freeze NCC_LOOP_LAG_MS=10 NCC_LOOP_LAG_FILE=$PWD/$out/cur_lag.jsonl python bench.py --steps 20 --warmup 5 --shard-latency-ms 5
