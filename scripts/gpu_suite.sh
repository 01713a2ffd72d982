#!/bin/bash
# GPU-box session: the five BASELINE configurations for one mode.  usage: gpu_suite.sh native|compat [extra args]
mode=${1:-native}; shift
mkdir -p gpurun_out
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 1050 python bench/suite.py --modes "$mode" --out gpurun_out/suite_$mode.json "$@" > gpurun_out/suite_$mode.log 2>&1
s=$?; echo "suite $mode: $s"; cat gpurun_out/suite_$mode.log | cut -c 1-400
