#!/bin/bash
# Executors-per-shard scan at N=1 (bench.py), one run per k; stops on the first fatal status.
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) echo "fatal status $1 in $2; stopping"; exit "$1";; esac; }
python native/build.py > gpurun_out/build.log 2>&1 || exit 1
for k in "$@"; do
  timeout -k 10 300 python bench.py --extra-env NEXUS__EXECUTORS_PER_SHARD=$k > gpurun_out/kscan_k$k.json 2> gpurun_out/kscan_k$k.err; s=$?; fatal $s k$k; echo "k=$k: $s"
done
tail -n 1 gpurun_out/kscan_k*.json
