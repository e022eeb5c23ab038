#!/bin/bash
# GPU session: shared-engine hub vs per-loop engines vs CPU engine (alternating).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/hub
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/hub/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/hub/gpu_tests.log; exit 1; }
tail -2 gpurun_out/hub/gpu_tests.log
run() {  # name, env..., args
  local name=$1; shift
  timeout -k 10 240 env "$@" > gpurun_out/hub/$name.json 2> gpurun_out/hub/$name.err || { echo "bench $name failed"; tail -20 gpurun_out/hub/$name.err; return 1; }
  echo "$name $(cat gpurun_out/hub/$name.json)"
}
for rep in 1 2; do
  run hip_shared_$rep QMX_SHARED_ENGINE=1 python bench.py --engine hip --steps 10 --warmup 2 &&
  run hip_perloop_$rep QMX_SHARED_ENGINE=0 python bench.py --engine hip --steps 10 --warmup 2 &&
  run cpu_$rep python bench.py --engine cpu --steps 10 --warmup 2 || exit 1
done
run hip_shared_t16 QMX_SHARED_ENGINE=1 python bench.py --engine hip --steps 10 --warmup 2 --threads 16 &&
run cpu_t16 python bench.py --engine cpu --steps 10 --warmup 2 --threads 16 || exit 1
echo "all done"
