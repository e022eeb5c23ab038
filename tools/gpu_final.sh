#!/bin/bash
# GPU session: GPU suite, smoke, headline bench x3 + scenarios, rocprof kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/final
mkdir -p $OUT/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err || { echo "bench failed"; tail -20 $OUT/bench_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$rep.json')); b=d.get('breakdown_one_rank',{}); print('bench', d['value'], d.get('p50_ttft_ms'), b.get('tick_kernel_us_avg'), b.get('proxy_cpu_ms_per_1k_req'))"
done
for SC in aggregate4 highqps8 failure; do
  timeout -k 10 300 python bench.py --scenario $SC --steps 10 --warmup 2 > $OUT/bench_$SC.json 2> $OUT/bench_$SC.err || { echo "bench $SC failed"; tail -20 $OUT/bench_$SC.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$SC.json')); print('$SC', d['value'], d.get('p50_ttft_ms'))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o native --output-format csv -- python3 bench.py --steps 5 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "prof failed"; tail -5 $OUT/bench_prof.err; exit 1; }
echo "all done"
