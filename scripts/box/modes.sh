#!/bin/bash
# Box: bench.py in native and compat-unthrottled mode (100 and 1000 templates), and both at 5 ms shard RTT.
set -o pipefail
out=${1:-gpurun_out/modes}
mkdir -p "$out"
b() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > $out/$name.json 2> $out/$name.err || exit $?
  python scripts/box/summarize.py $out/$name.json
}
b native_t100 --templates 100 --steps 10 --warmup 3
b unthrottled_t100 --mode compat-unthrottled --templates 100 --steps 10 --warmup 3
b unthrottled_t1000 --mode compat-unthrottled --steps 5 --warmup 2
b native_t100_lat5 --templates 100 --steps 10 --warmup 3 --shard-latency-ms 5
b unthrottled_t100_lat5 --mode compat-unthrottled --templates 100 --steps 3 --warmup 1 --shard-latency-ms 5
