#!/bin/bash
# The one box runner (replaces the per-session gpu_*.sh scripts of rounds 1-3).  Every step runs under its
# own time limit and the first failure ends the call.  Results go to gpurun_out/<out>/.
#
#   bash scripts/box/run.sh <out> tier                   GPU tier (pytest -m gpu) + smoke
#   bash scripts/box/run.sh <out> bench <n> [ARGS...]    the driver's bench shape n times; ARGS are bench.py
#                                                        flags or KEY=VAL environment for the controller
#   bash scripts/box/run.sh <out> ab <n> "<A>" "<B>"     A/B in alternation, n pairs; A and B are
#                                                        space-separated KEY=VAL lists ("-" = none)
#   bash scripts/box/run.sh <out> abtree <n> <dir>       this tree against another built tree (<dir>, e.g. an
#                                                        `abtree_*` copy shipped with the call), n pairs
#   bash scripts/box/run.sh <out> suite [suite.py args]  the five BASELINE.json configurations
#   bash scripts/box/run.sh <out> sweep [N...]           shards N (default 1 2 4; CPU ranks over gloo, torchrun) ×
#                                                        injected shard latency 0/5/20 ms, then 8 shards on one rank
#   bash scripts/box/run.sh <out> sample [steps]         sampling profiles of the C++ executor and the coordinator
#   bash scripts/box/run.sh <out> prof                   rocprofv3 --kernel-trace --stats over a short bench,
#                                                        and the C++ executor's own sampling profile
#   bash scripts/box/run.sh <out> modes                  native vs compat-unthrottled vs compat in one session,
#                                                        N=1 and 8 shards on one rank (reference-compat baseline)
#   bash scripts/box/run.sh <out> aimd [n]               AIMD vs NCC_AIMD=0 (fixed 256) in alternation, n pairs,
#                                                        shard RTT 5/20 ms × jitter 0/10/20 ms, N=1 and 8 shards
#   bash scripts/box/run.sh <out> http2 [n]              n rounds of: the driver shape over HTTP/1.1 and over HTTP/2
#                                                        (prior knowledge), then --tls over HTTP/1.1 and HTTP/2 (ALPN)
#   bash scripts/box/run.sh <out> ranks [N] [pairs]      torchrun with N CPU ranks (N shards), HTTP/1.1 vs HTTP/2
#   bash scripts/box/run.sh <out> multishard [n]         n rounds of: suite configs 2, 5, 8 with --stages, then
#                                                        bench.py N=1 and --shards-per-rank 8 --stages
#
# e.g.  gpurun -- 'bash scripts/box/run.sh r4a tier && bash scripts/box/run.sh r4a bench 3'
set -o pipefail
out=gpurun_out/$1
what=$2
shift 2
mkdir -p "$out"

summary() {  # one line per bench result
  python3 - "$1" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
h = d.get("host") or {}
c = h.get("calibration") or {}
print(sys.argv[1].split("/")[-1], d["value"], "p50", d["p50_latency_ms"], "p99", d["p99_latency_ms"],
      "ctl_us", d["controller_cpu_us_per_object"], d["controller_cpu_us_per_object_split"],
      "substrate_us", d.get("substrate_us_per_object"), "ratio", d.get("controller_to_substrate"),
      "coord_cores", d["cpu_cores_busy"].get("coordinator"), "py_loop_ms", c.get("python_loop_ms"),
      "cpp_scan_ns", c.get("cpp_ctl_scan_ns"), "throttled_us", h.get("throttled_usec"),
      "host_busy", h.get("host_busy_cpus"),
      "wakeups", ((d.get("controller_state") or {}).get("executor_flow") or {}).get("shard-0", {}).get("loop_wakeups"),
      "cold_s", d.get("cold_start_s"),
      "limit", ((d.get("controller_state") or {}).get("executor_flow") or {}).get("shard-0", {}).get("limit"),
      "held", ((d.get("controller_state") or {}).get("executor_flow") or {}).get("shard-0", {}).get("increases_held"),
      "h2", ((d.get("controller_state") or {}).get("executor_flow") or {}).get("shard-0", {}).get("http2"),
      "conns", ((d.get("controller_state") or {}).get("executor_flow") or {}).get("shard-0", {}).get("connections"),
      "ctl", (d.get("config") or {}).get("controller_transport"), flush=True)
EOF
}

bench_once() {  # <file> [ARGS...]
  local f=$1; shift
  local envs=() flags=() arg  # `arg` local: the ab preset's own $a / $b must survive this loop
  for arg in "$@"; do  # KEY=VAL: environment (bench.py passes it on to the controller); anything else: a flag
    if [[ "$arg" == *=* && "$arg" != -* ]]; then envs+=("$arg"); else flags+=("$arg"); fi
  done
  env "${envs[@]}" timeout -k 10 "${BENCH_TIMEOUT:-300}" python3 bench.py --gpus 1 --steps 20 --warmup 5 "${flags[@]}" \
    > "$f.json" 2> "$f.err" || return $?
  # a stderr holding nothing but the ROCm runtime's amdgpu.ids notice is not kept
  grep -qv 'amdgpu.ids: No such file' "$f.err" || rm -f "$f.err"
  summary "$f.json"
}

case "$what" in
  tier)
    timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > "$out/pytest_gpu.log" 2>&1 || { tail -30 "$out/pytest_gpu.log"; exit 1; }
    timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
      || { tail -30 "$out/smoke.log"; exit 1; }
    tail -1 "$out/pytest_gpu.log"; tail -1 "$out/smoke.log"
    ;;
  bench)
    n=$1; shift
    k=$(find "$out" -maxdepth 1 -name 'bench_*.json' | wc -l)  # a second `bench` into the same dir appends
    for i in $(seq $((k + 1)) $((k + n))); do bench_once "$out/bench_$i" "$@" || exit $?; done
    ;;
  ab)
    n=$1; a=$2; b=$3
    [ "$a" = "-" ] && a=""
    [ "$b" = "-" ] && b=""
    for i in $(seq 1 "$n"); do
      # shellcheck disable=SC2086
      bench_once "$out/a_$i" $a || exit $?
      # shellcheck disable=SC2086
      bench_once "$out/b_$i" $b || exit $?
    done
    ;;
  abtree)
    n=$1; other=$2
    for i in $(seq 1 "$n"); do
      bench_once "$out/head_$i" || exit $?
      (cd "$other" && bench_once "$OLDPWD/$out/other_$i") || exit $?
    done
    ;;
  sweep)
    ns=${*:-1 2 4}
    port=29710
    for n in $ns; do
      for lat in 0 5 20; do
        port=$((port + 1))
        f="$out/n${n}_lat${lat}"
        if [ "$n" = 1 ]; then
          bench_once "$f" --shard-latency-ms "$lat" || exit $?
        else
          timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
            --master-port "$port" bench.py --gpus "$n" --steps 20 --warmup 5 --shard-latency-ms "$lat" \
            > "$f.json" 2> "$f.err" || exit $?
          summary "$f.json"
        fi
      done
    done
    bench_once "$out/s8" --shards-per-rank 8 || exit $?
    ;;
  suite)
    timeout -k 10 900 python3 bench/suite.py --modes native --out "$out/suite.json" "$@" > "$out/suite.log" 2>&1 \
      || { tail -30 "$out/suite.log"; exit 1; }
    cut -c 1-300 "$out/suite.log" | tail -14
    ;;
  sample)  # the C++ executor's and the coordinator's sampling profiles over a long driver-shape run (args: steps, bench flags)
    # the frame-pointer build of the executor when it was built (native/build.py): call stacks in the profile
    exe=ncc/bin/ncc-executor
    [ -x build/profile/ncc-executor ] && exe=build/profile/ncc-executor
    NCC_EXECUTOR_BINARY="$PWD/$exe" \
    NCC_SAMPLE_PROFILE="$PWD/$out/samples" NCC_SAMPLE_US=200 NCC_PY_SAMPLE="$PWD/$out/py" NCC_PY_SAMPLE_US=200 \
      timeout -k 10 600 python3 bench.py --steps "${1:-100}" --warmup 5 "${@:2}" > "$out/sampled_bench.json" \
      2> "$out/sampled_bench.err" || exit $?
    python3 scripts/executor_profile.py "$out/samples" --binary "$exe" > "$out/executor_profile.txt" 2>&1 || true
    python3 scripts/py_profile.py "$out"/py.*.json > "$out/coordinator_profile.txt" 2>&1 || true
    summary "$out/sampled_bench.json"
    ;;
  prof)
    export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/rocprof" -o bench -- \
      python3 bench.py --steps 5 --warmup 2 > "$out/rocprof_bench.json" 2> "$out/rocprof.err" || exit $?
    NCC_SAMPLE_PROFILE="$PWD/$out/samples" NCC_SAMPLE_US=200 timeout -k 10 300 python3 bench.py --steps 20 \
      --warmup 5 > "$out/sampled_bench.json" 2> "$out/sampled_bench.err" || exit $?
    python3 scripts/executor_profile.py "$out/samples" > "$out/executor_profile.txt" 2>&1 || true
    python3 scripts/py_profile.py "$out"/py.*.json > "$out/coordinator_profile.txt" 2>&1 || true
    summary "$out/sampled_bench.json"
    ;;
  modes)
    # the reference's scheduling (sequential fail-fast shard loop, Event per reconcile, 2 workers) with and
    # without client-go's 5 QPS / burst 10, next to native, on one box in one session
    bench_once "$out/n1_native" || exit $?
    bench_once "$out/n1_unthrottled_t1000" --mode compat-unthrottled --steps 3 --warmup 1 || exit $?
    bench_once "$out/n1_native_t100" --templates 100 || exit $?
    # compat waves take ~40 s each: NCC_BENCH_DEBUG prints a line per wave (gpurun's idle watchdog sees it)
    BENCH_TIMEOUT=420 bench_once "$out/n1_compat_t100" NCC_BENCH_DEBUG=1 --mode compat --templates 100 --steps 2 \
      --warmup 1 || exit $?
    bench_once "$out/s8_native" --shards-per-rank 8 --steps 10 --warmup 3 || exit $?
    bench_once "$out/s8_unthrottled_t1000" --shards-per-rank 8 --mode compat-unthrottled --steps 2 --warmup 1 || exit $?
    bench_once "$out/s8_native_t100" --shards-per-rank 8 --templates 100 || exit $?
    BENCH_TIMEOUT=420 bench_once "$out/s8_compat_t50" NCC_BENCH_DEBUG=1 --shards-per-rank 8 --mode compat \
      --templates 50 --steps 1 --warmup 1 --timeout 400 || exit $?
    ;;
  aimd)
    n=${1:-1}
    for i in $(seq 1 "$n"); do
      for lat in 5 20; do
        for jit in 0 10 20; do
          for s in 1 8; do
            f="l${lat}_j${jit}_s${s}"
            bench_once "$out/${f}_aimd_$i" --shards-per-rank "$s" --shard-latency-ms "$lat" --shard-jitter-ms "$jit" \
              --steps 10 --warmup 3 || exit $?
            bench_once "$out/${f}_fixed_$i" NCC_AIMD=0 --shards-per-rank "$s" --shard-latency-ms "$lat" \
              --shard-jitter-ms "$jit" --steps 10 --warmup 3 || exit $?
          done
        done
      done
    done
    ;;
  coord)  # the coordinator's transport to the controller apiserver: HTTP/1.1 (a_) vs HTTP/2 (b_), executors on
           # HTTP/2 in both arms; cleartext and TLS (tls_a_, tls_b_)
    n=${1:-2}
    for i in $(seq 1 "$n"); do
      bench_once "$out/a_$i" NCC_HTTP2=2 NEXUS__CLIENT_HTTP2=off || exit $?
      bench_once "$out/b_$i" NCC_HTTP2=2 NEXUS__CLIENT_HTTP2=on || exit $?
      bench_once "$out/tls_a_$i" NCC_HTTP2=1 NEXUS__CLIENT_HTTP2=off --tls || exit $?
      bench_once "$out/tls_b_$i" NCC_HTTP2=1 NEXUS__CLIENT_HTTP2=auto --tls || exit $?
    done
    ;;
  http2)
    n=${1:-1}
    for i in $(seq 1 "$n"); do
      bench_once "$out/h1_$i" NEXUS__CLIENT_HTTP2=off || exit $?
      bench_once "$out/h2_$i" NEXUS__CLIENT_HTTP2=on || exit $?
      bench_once "$out/tls_h1_$i" NEXUS__CLIENT_HTTP2=off --tls || exit $?
      bench_once "$out/tls_h2_$i" --tls || exit $?
    done
    ;;
  ranks)  # torchrun over CPU ranks on this box (N shards, one per rank), HTTP/1.1 (a_) and HTTP/2 (b_) alternating
    n=${1:-2}; pairs=${2:-2}
    port=29740
    for i in $(seq 1 "$pairs"); do
      for arm in a b; do
        port=$((port + 1))
        h2=on; [ "$arm" = a ] && h2=off
        NEXUS__CLIENT_HTTP2=$h2 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
          --master-addr 127.0.0.1 --master-port "$port" bench.py --gpus "$n" --steps 20 --warmup 5 \
          > "$out/n${n}_${arm}_$i.json" 2> "$out/n${n}_${arm}_$i.err" || exit $?
        grep -qv 'amdgpu.ids: No such file' "$out/n${n}_${arm}_$i.err" || rm -f "$out/n${n}_${arm}_$i.err"
        summary "$out/n${n}_${arm}_$i.json"
      done
    done
    ;;
  multishard)
    n=${1:-1}
    for i in $(seq 1 "$n"); do
      timeout -k 10 600 python3 bench/suite.py --modes native --configs 2,5,8 --stages --out "$out/suite_$i.json" \
        > "$out/suite_$i.log" 2>&1 || { tail -30 "$out/suite_$i.log"; exit 1; }
      cut -c 1-400 "$out/suite_$i.log" | grep '^{'
      bench_once "$out/n1_$i" --stages || exit $?
      bench_once "$out/s8_$i" --shards-per-rank 8 --stages || exit $?
    done
    ;;
  *)
    echo "unknown preset $what" >&2; exit 2;;
esac
