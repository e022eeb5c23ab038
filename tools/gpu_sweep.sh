#!/bin/bash
# GPU session: headline bench over connections per rank (and tick lanes), two reps each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/sweep
mkdir -p $OUT
run() {  # name, env..., args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); b=d['breakdown_one_rank']; print('$name', d['value'], d['p50_ttft_ms'], d['p99_ttft_ms'], b.get('streams_per_tick'), b.get('tick_wall_us_avg'), b.get('tick_kernel_us_avg'), b.get('gpu_busy_frac'), b.get('proxy_cpu_ms_per_1k_req'), b.get('cores_busy'))"
}
for rep in 1 2; do
  for c in 64 96 128 192 256; do
    run c${c}_$rep python bench.py --conns $c || exit 1
  done
  run c128_l3_$rep QMX_TICK_LANES=3 python bench.py --conns 128 || exit 1
done
echo "all done"
