#!/bin/bash
# GPU-box session: native build, `pytest -m gpu`, bench at N=1 and CPU-rank rehearsals at N=2,4
# (ranks only call torch.cuda.synchronize on device 0; the 8-GPU scaling run is the driver's).
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; s=$?; fatal $s pytest; echo "pytest gpu: $s"
NCC_BENCH_DEBUG=1 timeout -k 10 600 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err; s=$?; fatal $s bench1; echo "bench n1: $s"
for n in 2 4; do
  NCC_BENCH_DEBUG=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2960$n \
    bench.py --gpus $n > gpurun_out/bench_n$n.json 2> gpurun_out/bench_n$n.err; s=$?; fatal $s bench$n; echo "bench n$n: $s"
done
tail -n 1 gpurun_out/bench_n*.json
