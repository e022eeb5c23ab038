#!/bin/bash
# GPU session: tick kernel with 1024-thread workgroups — correctness + stage timing + bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/bs
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
QMX_STAGE_TIMING=1 timeout -k 10 200 python tools/kbench.py --slots 1,64,256 --iters 20 > $OUT/kbench.jsonl 2>&1 || { echo "kbench failed"; tail -5 $OUT/kbench.jsonl; exit 1; }
python3 -c "
import json
for l in open('$OUT/kbench.jsonl'):
    if not l.startswith('{'): continue
    d=json.loads(l); st=d.get('stage_us_per_item',{})
    print(d['filter'],d['emit'],d['slots'],d['wall_us_p50'],d['kernel_us_avg'],[st.get('stage%d_us'%k) for k in range(1,11)])
"
for rep in 1 2; do
  timeout -k 10 240 python bench.py --steps 10 --warmup 2 > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err || { echo "bench failed"; tail -20 $OUT/bench_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$rep.json')); b=d['breakdown_one_rank']; print('bench', d['value'], d['p50_ttft_ms'], b.get('tick_kernel_us_avg'), b.get('tick_wall_us_avg'), b.get('proxy_cpu_ms_per_1k_req'))"
done
echo "all done"
