#!/bin/bash
# GPU session: tests, headline bench, BASELINE scenario benches, kernel microbench,
# rocprof kernel stats and PMC counters (separate runs: --pmc never with tracing).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/pmc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
for SC in aggregate4 highqps8 failure; do
  timeout -k 10 300 python bench.py --scenario $SC --steps 10 --warmup 2 > gpurun_out/bench_$SC.json 2> gpurun_out/bench_$SC.err || { echo "bench $SC failed"; tail -20 gpurun_out/bench_$SC.err; exit 1; }
  cat gpurun_out/bench_$SC.json
done
QMX_STAGE_TIMING=1 timeout -k 10 300 python tools/kbench.py --slots 1,64,256,1024 --iters 20 > gpurun_out/kbench.jsonl 2>&1 || { echo "kbench failed"; tail -5 gpurun_out/kbench.jsonl; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o native --output-format csv -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || { echo "prof failed"; tail -5 gpurun_out/bench_prof.err; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_I8 SQ_INSTS_VALU_MFMA_MOPS_I8 --kernel-trace --stats -d gpurun_out/pmc -o pmc1 --output-format csv -- python3 tools/kbench.py --slots 256 --iters 10 > gpurun_out/pmc1.log 2>&1 || { echo "pmc1 failed"; tail -5 gpurun_out/pmc1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --stats -d gpurun_out/pmc -o pmc2 --output-format csv -- python3 tools/kbench.py --slots 256 --iters 10 > gpurun_out/pmc2.log 2>&1 || { echo "pmc2 failed"; tail -5 gpurun_out/pmc2.log; exit 1; }
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d gpurun_out/prof -o markers --output-format csv -- python3 bench.py --steps 2 --warmup 1 --batch 2048 > gpurun_out/bench_markers.json 2> gpurun_out/bench_markers.err || { echo "marker trace failed"; tail -5 gpurun_out/bench_markers.err; exit 1; }
echo "all done"
