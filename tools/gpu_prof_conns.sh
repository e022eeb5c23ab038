#!/bin/bash
# GPU session: in-process CPU profile of the proxy at 64 vs 128 connections per rank.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/profc
mkdir -p $OUT
for c in 64 128; do
  timeout -k 10 240 env QMX_PROF=$PWD/$OUT/cpu_c$c.%p.txt python bench.py --conns $c --steps 30 > $OUT/c$c.json 2> $OUT/c$c.err || { echo "bench c$c failed"; tail -20 $OUT/c$c.err; exit 1; }
  python3 tools/cpuprof.py --top 40 $OUT/cpu_c$c.*.txt > $OUT/summary_c$c.txt || exit 1
done
echo "all done"
