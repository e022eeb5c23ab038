#!/bin/bash
# GPU session: headline bench A/B (HIP hub 1 / 2 tick lanes vs C++ CPU engine), 3 reps,
# plus a CPU profile of the HIP path; GPU tests first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/ab
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
run() {  # name, env..., args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); b=d['breakdown_one_rank']; print('$name', d['value'], d['p50_ttft_ms'], d['p99_ttft_ms'], b.get('streams_per_tick'), b.get('tick_wall_us_avg'), b.get('tick_kernel_us_avg'), b.get('tick_launch_wait_us_avg'), b.get('proxy_cpu_ms_per_1k_req'), b.get('mocks_cpu_ms_per_1k_req'), b.get('loadgen_cpu_ms_per_1k_req'))"
}
for rep in 1 2 3; do
  run l1_$rep QMX_TICK_LANES=1 python bench.py --steps 10 --warmup 2 &&
  run l2_$rep QMX_TICK_LANES=2 python bench.py --steps 10 --warmup 2 &&
  run cpu_$rep python bench.py --engine cpu --steps 10 --warmup 2 || exit 1
done
run prof_l1 QMX_PROF=$PWD/$OUT/cpu_l1.%p.txt QMX_TICK_LANES=1 python bench.py --steps 20 --warmup 2 || exit 1
echo "all done"
