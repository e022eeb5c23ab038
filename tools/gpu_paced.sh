#!/bin/bash
# GPU session: GPU tests + the paced (steady-state streaming) scenario, HIP vs CPU engine.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/paced
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
run() {  # name, env..., args
  local name=$1; shift
  timeout -k 10 240 env "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); b=d['breakdown_one_rank']; print('$name', d['value'], d['p50_ttft_ms'], d['p99_ttft_ms'], d['p50_latency_ms'], d['errors'], b.get('streams_per_tick'), b.get('tick_wall_us_avg'), b.get('tick_kernel_us_avg'), b.get('proxy_cpu_ms_per_1k_req'), b.get('cores_busy'))"
}
run paced_hip python bench.py --scenario paced --steps 4 --warmup 1 --batch 4096 &&
run paced_cpu python bench.py --scenario paced --engine cpu --steps 4 --warmup 1 --batch 4096 &&
run paced_hip_4k python bench.py --scenario paced --steps 4 --warmup 1 --batch 8192 --conns 4096 &&
run paced_cpu_4k python bench.py --scenario paced --engine cpu --steps 4 --warmup 1 --batch 8192 --conns 4096 || exit 1
echo "all done"
