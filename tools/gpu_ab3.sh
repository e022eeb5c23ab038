#!/bin/bash
# GPU session: interleaved A/B of load-generator threads (2 vs 4) and tick lanes (2 vs 3) at 64 conns.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/ab3
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  timeout -k 10 240 env "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); b=d['breakdown_one_rank']; print('$name', d['value'], d['p50_ttft_ms'], b.get('streams_per_tick'), b.get('tick_wall_us_avg'), b.get('gpu_busy_frac'), b.get('proxy_cpu_ms_per_1k_req'), b.get('cores_busy'))"
}
for rep in 1 2 3 4 5; do
  run lg2_$rep python bench.py --lg-threads 2 || exit 1
  run lg4_$rep python bench.py --lg-threads 4 || exit 1
  run lg4_l3_$rep QMX_TICK_LANES=3 python bench.py --lg-threads 4 || exit 1
done
echo "all done"
