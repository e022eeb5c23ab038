#!/bin/bash
# GPU session: loop wake-up only when parked (default) vs an eventfd write per result batch (QMX_EVFD_ALWAYS=1), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/ab5
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  timeout -k 10 240 env "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); b=d['breakdown_one_rank']; print('$name', d['value'], d['p50_ttft_ms'], d.get('p50_ttfb_ms'), b.get('streams_per_tick'), b.get('gpu_busy_frac'), b.get('proxy_cpu_ms_per_1k_req'), b.get('loadgen_cpu_ms_per_1k_req'), b.get('cores_busy'))"
}
timeout -k 10 300 python -u -m pytest tests/test_gpu_native_server.py -x -q --timeout 120 --timeout-method thread > $OUT/gpu_server_tests.log 2>&1 || { echo "gpu server tests failed"; tail -30 $OUT/gpu_server_tests.log; exit 1; }
tail -1 $OUT/gpu_server_tests.log
for rep in 1 2 3 4 5; do
  run always_$rep QMX_EVFD_ALWAYS=1 python bench.py || exit 1
  run on_$rep python bench.py || exit 1
done
echo "all done"
