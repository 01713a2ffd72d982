#!/bin/bash
# Heavy chaos exploration and the CPU test tier on the box.  Usage: bash scripts/gpu_r3_chaos.sh <dir>
out=gpurun_out/$1
mkdir -p $out
NCC_CHAOS_STEPS=200 NCC_CHAOS_SEEDS=24 NCC_CHAOS_KILLS=4 timeout -k 10 400 python3 -m pytest tests/test_chaos.py -q -n 8 -p no:cacheprovider > $out/chaos.log 2>&1
echo "chaos=$?"; tail -2 $out/chaos.log
timeout -k 10 400 python3 -m pytest tests -q -m "not gpu" -n 8 -p no:cacheprovider > $out/cpu_suite.log 2>&1
echo "suite=$?"; tail -2 $out/cpu_suite.log
