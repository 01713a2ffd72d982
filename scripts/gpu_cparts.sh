#!/bin/bash
# Coordinator partitions on the 1-GPU box: 8 shard apiservers on one rank, C = 1 / 2 / 3.
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
for r in 1 2; do for C in 1 2; do
  timeout -k 10 300 python bench.py --shards-per-rank 8 --extra-env NEXUS__COORDINATOR_PARTITIONS=$C \
    > gpurun_out/cp_${C}_$r.json 2>gpurun_out/cp_${C}_$r.err; s=$?; fatal $s c$C
  python -c "
import json; d=json.loads(open('gpurun_out/cp_${C}_$r.json').read().strip().splitlines()[-1]); c=d['cpu_cores_busy']
print('C=$C', d['value'], d['p50_latency_ms'], d['p99_latency_ms'], c)"
done; done
