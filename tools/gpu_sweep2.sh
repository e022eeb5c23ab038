#!/bin/bash
# GPU session: is the harness (load generator / mocks) the bound?  lg-threads x mock-threads x conns.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/sweep2
mkdir -p $OUT
run() {  # name, args
  local name=$1; shift
  timeout -k 10 240 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); b=d['breakdown_one_rank']; print('$name', d['value'], d['p50_ttft_ms'], b.get('streams_per_tick'), b.get('tick_wall_us_avg'), b.get('gpu_busy_frac'), b.get('proxy_cpu_ms_per_1k_req'), b.get('cores_busy'))"
}
for rep in 1 2; do
  run lg2_m2_c64_$rep --lg-threads 2 --mock-threads 2 --conns 64 || exit 1
  run lg4_m2_c64_$rep --lg-threads 4 --mock-threads 2 --conns 64 || exit 1
  run lg4_m4_c64_$rep --lg-threads 4 --mock-threads 4 --conns 64 || exit 1
  run lg4_m4_c128_$rep --lg-threads 4 --mock-threads 4 --conns 128 || exit 1
  run lg6_m4_c128_$rep --lg-threads 6 --mock-threads 4 --conns 128 || exit 1
  run lg4_m4_c96_t10_$rep --lg-threads 4 --mock-threads 4 --conns 96 --threads 10 || exit 1
done
echo "all done"
