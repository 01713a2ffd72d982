#!/bin/bash
# Box: the automatic sizing a large node picks (NCC_CPU_SHARE=128 -> 4 coordinators x k=4 executors per
# shard), rehearsed with 4 torchrun ranks on the 1-GPU box (the driver's 8-rank run is not ours to start).
set -o pipefail
out=${1:-gpurun_out/bignode}
mkdir -p "$out"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29631 bench.py --gpus 4 --steps 20 --warmup 5 --extra-env NCC_CPU_SHARE=128 \
  > $out/n4_share128.json 2> $out/n4_share128.err || exit $?
python scripts/box/summarize.py $out/n4_share128.json
python -c "import json;d=json.loads(open('$out/n4_share128.json').read().strip().splitlines()[-1]);print(d['controller_sizing'], d['controller_children'], d['controller_apiserver_load'])"
