#!/bin/bash
# GPU session: GPU tests, then headline bench HIP (x3) vs CPU engine (x2), CPU profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/ab2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
run() {  # name, env..., args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); b=d['breakdown_one_rank']; print('$name', d['value'], d['p50_ttft_ms'], d['p99_ttft_ms'], b.get('streams_per_tick'), b.get('tick_wall_us_avg'), b.get('tick_kernel_us_avg'), b.get('tick_host_prep_us_avg'), b.get('tick_launch_wait_us_avg'), b.get('tick_process_us_avg'), b.get('proxy_cpu_ms_per_1k_req'))"
}
for rep in 1 2 3; do
  run hip_$rep python bench.py --steps 10 --warmup 2 && run hip_l2_$rep QMX_TICK_LANES=2 python bench.py --steps 10 --warmup 2 || exit 1
  if [ $rep -le 2 ]; then run cpu_$rep python bench.py --engine cpu --steps 10 --warmup 2 || exit 1; fi
done
run prof QMX_PROF=$PWD/$OUT/cpu_hip.%p.txt python bench.py --steps 30 --warmup 2 || exit 1
echo "all done"
