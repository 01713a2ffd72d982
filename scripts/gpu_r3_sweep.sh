#!/bin/bash
# round-3 box sweep: N=1/2/4 (CPU ranks over gloo; one shard apiserver per rank) x injected shard latency
# 0/5/20 ms, native defaults; then 8 shards on one rank.  Usage: bash scripts/gpu_r3_sweep.sh <out dir name>
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
port=29710
run() {  # name, nproc, args...
  local name=$1 n=$2; shift 2
  port=$((port + 1))
  if [ "$n" = "1" ]; then
    timeout -k 10 300 python3 bench.py "$@" > $out/$name.json 2> $out/$name.err || return $?
  else
    timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus $n "$@" > $out/$name.json 2> $out/$name.err || return $?
  fi
  python3 -c "import json;d=json.loads([l for l in open('$out/$name.json').read().splitlines() if l.startswith('{')][-1]);print('$name',d['value'],d['p50_latency_ms'],d['p99_latency_ms'],d['controller_cpu_us_per_object'],d['controller_cpu_us_per_object_split'],d['controller_sizing'].get('coordinator_partitions'),d.get('controller_children'),flush=True)"
}
for n in 1 2 4; do
  for lat in 0 5 20; do
    run n${n}_lat${lat} $n --steps 20 --warmup 5 --shard-latency-ms $lat || exit $?
  done
done
run s8 1 --shards-per-rank 8 --steps 20 --warmup 5 || exit $?
