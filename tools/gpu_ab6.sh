#!/bin/bash
# GPU session: scenarios (highqps8, aggregate4) with role deferral / loop wake-up variants, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/ab6
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  timeout -k 10 240 env "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); b=d['breakdown_one_rank']; print('$name', d['value'], d['p50_ttft_ms'], b.get('streams_per_tick'), b.get('gpu_busy_frac'), b.get('proxy_cpu_ms_per_1k_req'), b.get('cores_busy'))"
}
for rep in 1 2 3; do
  for SC in highqps8 aggregate4; do
    run ${SC}_default_$rep python bench.py --scenario $SC --steps 10 --warmup 2 || exit 1
    run ${SC}_nodefer_$rep QMX_ROLE_DEFER_US=0 python bench.py --scenario $SC --steps 10 --warmup 2 || exit 1
    run ${SC}_nodefer_evfd_$rep QMX_ROLE_DEFER_US=0 QMX_EVFD_ALWAYS=1 python bench.py --scenario $SC --steps 10 --warmup 2 || exit 1
  done
done
echo "all done"
