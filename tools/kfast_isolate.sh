#!/bin/bash
# Which single-wave fast path (QMX_KFAST bit) changes the HIP engine's output?  Runs the
# HIP-vs-CPU differential tests under each mask; stops at anything worse than a failed test.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/kfast
for m in ${@:-0 1 2 4 8 15}; do
  QMX_KFAST=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -x -q --timeout 120 \
    --timeout-method thread -k "wide_tags or matches_cpu_random" > gpurun_out/kfast/kfast_$m.log 2>&1
  rc=$?
  echo "KFAST=$m rc=$rc $(tail -1 gpurun_out/kfast/kfast_$m.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: rc $rc"; exit $rc; fi
done
