#!/bin/bash
# Box sweep: shards N=1/2/4 (one rank per GPU slot, torchrun CPU ranks) x injected shard latency 0/5/20 ms.
# usage: bash scripts/box/latency_sweep.sh <outdir>
set -o pipefail
out=${1:-gpurun_out/sweep}
mkdir -p "$out"
port=29610
for n in 1 2 4; do
  for lat in 0 5 20; do
    name=n${n}_lat${lat}
    if [ "$n" = 1 ]; then
      timeout -k 10 300 python bench.py --steps 20 --warmup 5 --shard-latency-ms $lat > $out/$name.json 2> $out/$name.err || exit $?
    else
      port=$((port + 1))
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
        --master-port $port bench.py --gpus $n --steps 20 --warmup 5 --shard-latency-ms $lat \
        > $out/$name.json 2> $out/$name.err || exit $?
    fi
    python scripts/box/summarize.py $out/$name.json
  done
done
