#!/bin/bash
# Where do the tick kernel's wave-cycles go?  Lists the box's counters, then one rocprofv3
# --pmc pass (instruction-cache and wait counters that exist on this GPU, at most 8 SQ) on
# kbench, summarised to gpurun_out/pmc_icache/summary.md.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmc_icache
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1
want=""
n=0
for c in SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES; do
  if grep -q "\b$c\b" $OUT/list_avail.txt; then want="$want $c"; n=$((n+1)); fi
done
echo "counters:$want"
[ -n "$want" ] || exit 0
QMX_PERSISTENT=0 timeout -s KILL 120 rocprofv3 --pmc $want -d $OUT/raw -o pmc --output-format csv -- \
  python3 tools/kbench.py --slots 22 --iters 10 > $OUT/kbench.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/kbench.log; exit 1; }
python3 tools/pmc_summary.py $(find $OUT/raw -name '*counter_collection.csv') > $OUT/summary.md 2>&1
grep "qmx_tick" $OUT/summary.md
