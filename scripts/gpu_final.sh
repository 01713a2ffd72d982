#!/bin/bash
# Round-end style verification on the box: build, pytest -m gpu, smoke, bench N=1 (+N=2, N=4), rocprofv3 kernel trace.
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; s=$?; fatal $s pytest; echo "pytest gpu: $s"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; s=$?; fatal $s smoke; echo "smoke: $s"; tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/final_n1.json 2>/dev/null; s=$?; fatal $s n1
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port 2960$n bench.py --gpus $n > gpurun_out/final_n$n.json 2>/dev/null; s=$?; fatal $s n$n
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof -o bench -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/rocprof_bench.json 2> gpurun_out/rocprof.log; s=$?; echo "rocprof: $s"
for f in gpurun_out/final_n*.json; do python -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['cold_start_s'])"; done
find gpurun_out/rocprof -type f | head
