#!/bin/bash
# A/B (ab_old vs current tree, N=1, alternating) + one N=1 run with per-wave phase timings (NCC_BENCH_DEBUG).
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
bash scripts/gpu_ab.sh "$@" || exit $?
NCC_BENCH_DEBUG=1 timeout -k 10 300 python bench.py "$@" > gpurun_out/debug_n1.json 2> gpurun_out/debug_n1.err; s=$?; fatal $s debug
grep "^#" gpurun_out/debug_n1.err | tail -12
