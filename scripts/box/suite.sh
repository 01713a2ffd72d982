#!/bin/bash
# Box run of the five BASELINE.json configurations: native and compat-unthrottled (reference scheduling
# without client-go's 5 QPS / 10 burst limiter).  usage: bash scripts/box/suite.sh <outdir>
set -o pipefail
out=${1:-gpurun_out/suite}
mkdir -p "$out"
timeout -k 10 420 python -u bench/suite.py --modes native --timeout 200 --out $out/suite_native.json \
  > $out/suite_native.log 2>&1 || exit $?
timeout -k 10 700 python -u bench/suite.py --modes compat-unthrottled --timeout 240 \
  --out $out/suite_compat_unthrottled.json > $out/suite_compat_unthrottled.log 2>&1 || exit $?
