#!/bin/bash
# GPU session: tick lanes sweep (1/2/3 kernels in flight) vs the C++ CPU engine, with the
# per-component CPU breakdown; GPU test suite first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/lanes
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
run() {  # name, env..., args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); b=d['breakdown_one_rank']; print('$name', d['value'], d['p50_ttft_ms'], d['p99_ttft_ms'], b.get('streams_per_tick'), b.get('tick_wall_us_avg'), b.get('tick_kernel_us_avg'), b.get('cores_busy'))"
}
for rep in 1 2; do
  run l1_$rep QMX_TICK_LANES=1 python bench.py --steps 10 --warmup 2 &&
  run l2_$rep QMX_TICK_LANES=2 python bench.py --steps 10 --warmup 2 &&
  run l3_$rep QMX_TICK_LANES=3 python bench.py --steps 10 --warmup 2 &&
  run cpu_$rep python bench.py --engine cpu --steps 10 --warmup 2 || exit 1
done
run l2_c128 QMX_TICK_LANES=2 python bench.py --steps 10 --warmup 2 --conns 128 &&
run cpu_c128 python bench.py --engine cpu --steps 10 --warmup 2 --conns 128 &&
run l2_c32 QMX_TICK_LANES=2 python bench.py --steps 10 --warmup 2 --conns 32 || exit 1
echo "all done"
