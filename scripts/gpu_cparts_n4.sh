#!/bin/bash
# N=4 ranks on the 1-GPU box: coordinator partitions C=1 vs C=2 (executors per shard fixed at 2 and 4 so k/C is whole).
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
for r in 1 2; do for cfg in "1 2" "2 2" "1 3"; do set -- $cfg; C=$1; K=$2
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 2950$C bench.py --gpus 4 --extra-env NEXUS__COORDINATOR_PARTITIONS=$C --extra-env NEXUS__EXECUTORS_PER_SHARD=$K \
    > gpurun_out/c4_${C}_${K}_$r.json 2>/dev/null; s=$?; fatal $s c$C
  python -c "
import json; d=json.loads(open('gpurun_out/c4_${C}_${K}_$r.json').read().strip().splitlines()[-1]); c=d['cpu_cores_busy']
print('N=4 C=$C k=$K', d['value'], d['p50_latency_ms'], c['coordinator'], c['executors'])"
done; done
