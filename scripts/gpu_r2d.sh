#!/bin/bash
# round-2 box sweep: N=1/2/4 (CPU ranks over gloo; one shard apiserver per rank) x injected shard latency
# 0/5/20 ms, native defaults; the three-mode baseline at N=1; 8 shards (4 ranks x 2) with C=1 vs forced C=4
set -o pipefail
out=gpurun_out/r2d
mkdir -p $out
port=29610
run() {  # name, nproc, args...
  local name=$1 n=$2; shift 2
  port=$((port + 1))
  if [ "$n" = "1" ]; then
    timeout -k 10 300 python bench.py "$@" > $out/$name.json 2> $out/$name.err || return $?
  else
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus $n "$@" > $out/$name.json 2> $out/$name.err || return $?
  fi
  python -c "import json;d=json.loads([l for l in open('$out/$name.json').read().splitlines() if l.startswith('{')][-1]);print('$name',d['value'],d['p50_latency_ms'],d['p99_latency_ms'],d['controller_cpu_us_per_object'],d['controller_cpu_us_per_object_split'],d['controller_sizing'].get('coordinator_partitions'),d.get('controller_children'))"
}
for n in 1 2 4; do
  for lat in 0 5 20; do
    run n${n}_lat${lat} $n --steps 20 --warmup 5 --shard-latency-ms $lat || exit $?
  done
done
run n1_compat_unthrottled 1 --mode compat-unthrottled --steps 5 --warmup 2 || exit $?
run n1_compat 1 --mode compat --templates 100 --steps 2 --warmup 1 || exit $?
run s8_c1 4 --shards-per-rank 2 --steps 10 --warmup 3 || exit $?
run s8_c4 4 --shards-per-rank 2 --steps 10 --warmup 3 --extra-env NCC_CPU_SHARE=128 || exit $?
