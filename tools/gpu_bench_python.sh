#!/bin/bash
# GPU box: python-impl bench with the HIP engine + rocprofv3 kernel stats of one short run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 400 python bench.py --impl python --engine hip --steps 10 --warmup 2 --batch 500 --conns 64 --workers 6 > gpurun_out/bench_python_hip.json 2> gpurun_out/bench_python_hip.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --impl python --engine hip --steps 2 --warmup 1 --batch 300 --conns 64 --workers 1 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
echo "rc=$?"
find gpurun_out/prof -name "*stats*" | head
