#!/bin/bash
# Mid-round GPU check: topology probe, GPU suite, headline bench x2, rocprof kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/check
mkdir -p $OUT/prof
timeout -k 10 120 python -c "
import torch
from quorum_amd.parallel import topology as t
p = torch.cuda.get_device_properties(0)
print('kfd numa', t.gpu_numa_nodes(), 'torch pci', p.pci_domain_id, p.pci_bus_id, p.pci_device_id,
      'numa', t.pci_numa_node(p.pci_domain_id, p.pci_bus_id, p.pci_device_id), 'summary', t.summary())
" > $OUT/topo.log 2>&1 || { echo "topo failed"; tail -20 $OUT/topo.log; exit 1; }
cat $OUT/topo.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err || { echo "bench failed"; tail -20 $OUT/bench_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$rep.json')); b=d.get('breakdown_one_rank',{}); print('bench', d['value'], d.get('p50_ttft_ms'), b.get('tick_wall_us_avg'), b.get('tick_kernel_us_avg'), b.get('tick_host_prep_us_avg'), b.get('proxy_cpu_ms_per_1k_req'))"
done
echo "all done"
