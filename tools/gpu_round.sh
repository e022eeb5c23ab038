#!/bin/bash
# One GPU-box session: gpu tests, native+hip bench, kernel microbench, rocprof kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
for T in 4 8; do
  timeout -k 10 300 python bench.py --threads $T --conns 256 --batch 4000 --steps 10 --lg-threads 4 --mock-threads 4 > gpurun_out/bench_t$T.json 2> gpurun_out/bench_t$T.err || { echo "bench t$T failed"; tail -20 gpurun_out/bench_t$T.err; exit 1; }
  cat gpurun_out/bench_t$T.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o native --output-format csv -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
echo "prof rc=$?"
