#!/bin/bash
# GPU session: does a longer timed window (requests per step) steady the headline number?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/batch
mkdir -p $OUT
run() {  # name, args
  local name=$1; shift
  timeout -k 10 240 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "bench $name failed"; tail -20 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/$name.json')); b=d['breakdown_one_rank']; print('$name', d['value'], d['ms_per_step'], d['p50_ttft_ms'], b.get('streams_per_tick'), b.get('gpu_busy_frac'), b.get('proxy_cpu_ms_per_1k_req'), d['config'].get('cpu_pinning'))"
}
for rep in 1 2 3 4; do
  run b4k_$rep || exit 1
  run b16k_$rep --batch 16384 || exit 1
done
echo "all done"
