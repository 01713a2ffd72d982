#!/bin/bash
# Box: eight shards on one rank with coordinator partitions C=2/3/4 (shared executors) in alternation;
# cpu_cores_busy reports the parent coordinator alone as `coordinator-parent`.
set -o pipefail
out=${1:-gpurun_out/spr8_c234}
mkdir -p "$out"
for i in 1 2; do
  for c in 2 3 4; do
    timeout -k 10 300 python bench.py --shards-per-rank 8 --steps 20 --warmup 5 \
      --extra-env NEXUS__COORDINATOR_PARTITIONS=$c > $out/c${c}_$i.json 2> $out/c${c}_$i.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); b=d['cpu_cores_busy']; print(sys.argv[1], d['value'], d['p50_latency_ms'], {k: b.get(k) for k in ('coordinator', 'coordinator-parent', 'executors', 'shard-apiserver', 'controller-apiserver')})" $out/c${c}_$i.json
  done
done
