#!/bin/bash
# One GPU-box session: box info, native build, `pytest -m gpu`, bench at N=1 (native + compat).
# Each step has its own time limit; a hard failure (timeout/abort/segfault) ends the script.
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
(nproc; lscpu | head -20; free -g; rocm-smi --showproductname 2>&1 | head -20) > gpurun_out/box_info.txt 2>&1
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; s=$?; fatal $s pytest; echo "pytest gpu: $s"
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err; s=$?; fatal $s bench; echo "bench: $s"
timeout -k 10 600 python bench.py --mode compat --templates 100 --steps 2 --warmup 1 > gpurun_out/bench_n1_compat.json 2> gpurun_out/bench_n1_compat.err; s=$?; fatal $s bench-compat; echo "bench compat: $s"
cat gpurun_out/bench_n1.json gpurun_out/bench_n1_compat.json
