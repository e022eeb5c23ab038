#!/bin/bash
# GPU session: rehearse the driver's multi-rank bench on a 1-GPU box (ranks share GPU 0;
# the bench's bookkeeping group falls back to gloo): 2 and 4 ranks, local placement, and
# 2 ranks with spread placement over the TCP exchange.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/multirank
mkdir -p $OUT
python3 -c "from quorum_amd.parallel.topology import summary; print('topology', summary())"
ls /sys/class/kfd/kfd/topology/nodes 2>&1 | head -3
tr() {  # name nproc args...
  local name=$1 np=$2; shift 2
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 500)) bench.py --gpus $np "$@" > $OUT/$name.out 2> $OUT/$name.err || { echo "$name failed"; tail -30 $OUT/$name.err; return 1; }
  grep '"metric"' $OUT/$name.out | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); b=d['breakdown_one_rank']; print('$name', d['value'], d['n_gpus'], d['p50_ttft_ms'], d['errors'], d['config']['parallelism'], b.get('exchange_rounds'))"
}
tr r2 2 --steps 5 --warmup 1 &&
tr r4 4 --steps 5 --warmup 1 --threads 4 &&
QMX_XCHG=tcp tr r2_spread 2 --steps 5 --warmup 1 --placement spread || exit 1
echo "all done"
