#!/bin/bash
# One parameterised MI355X session for gpurun: each argument is a step, run in order, each
# under its own time limit; the first failing step ends the session (no retries, nothing
# else touches the GPU after a fault / abort / timeout).
#
#   gpurun -- 'bash tools/gpu_session.sh TAG step [step ...]'
#
# steps:
#   tests                 pytest -m gpu (HIP engine vs C++ oracle, HIP server with verify mode)
#   pytest:F1,F2          selected GPU test files only
#   envtests:V=X,...      the whole GPU suite under extra env
#   smoke                 __graft_entry__.smoke()
#   bench[=N]             headline bench.py N times (default 1)            -> bench_<i>.json
#   bench:ARGS            one bench.py run with extra args (commas = spaces) -> bench_<slug>.json
#   hunt=N                N headline runs that go on past an invalid one; whole invalid bodies
#                         -> invalid_bodies.txt (QMX_LOADGEN_DUMP)
#   ab:NAME:ENV:ARGS      one bench.py run under extra env (commas = spaces) -> ab_<NAME>.json
#   scenarios             aggregate4, highqps8, failure, paced, nonstream1, direct (10 steps each)
#   reference             the upstream proxy under the same harness (bench.py --impl reference)
#   refscenarios          the same for nonstream1, aggregate4, highqps8, failure
#   prof                  rocprofv3 --kernel-trace --stats of a short headline bench
#   pmc:C1,C2,...         rocprofv3 --pmc pass (one block-limited counter set) on kbench
#   pmce:ENV=V:C1,C2      the same pass under extra env (e.g. QMX_KFAST=7: one fast path off)
#   pmcgrid:C1,C2,...     rocprofv3 --pmc on the production kernel (kbench --grid: qmx_tick_persistent),
#                         counters per dispatch and per tick (KB_GRID doors, default 16; KB_SLOTS streams)
#   kbench                tools/kbench.py in-kernel stage split (QMX_STAGE_TIMING)
#   kbenchgrid            the same on the persistent grid (the production kernel)
#   kbenchshape:SHAPE     the grid stage split on another stream shape (tools/kbench.py --shape: tagdense)
#   pmcshape:SHAPE:C,...  rocprofv3 --pmc on the production kernel for that shape, per tick
#   multirank=N           bench.py under torch.distributed.run with N ranks sharing GPU 0
#   spread=N              same, --placement spread over the TCP exchange
#   cpuprof               headline bench with the in-process CPU profiler on the proxy
#   cpuprofsc:SCENARIO    the same for a scenario (aggregate4, highqps8, failure, ...)
#   probe:NAME            tools/probes/NAME (built beforehand), e.g. probe:doorbell_probe
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT/prof

summ() {  # one line per bench JSON
  python3 - "$1" "$2" <<'EOF'
import json, sys
name, path = sys.argv[1], sys.argv[2]
lines = [l for l in open(path) if l.startswith("{")]
if not lines:
    print(name, "no JSON line"); sys.exit(0)
d = json.loads(lines[-1]); b = d.get("breakdown_one_rank", {})
print(name, d["value"], "p50ttft", d.get("p50_ttft_ms"), "valid", d.get("valid"), d.get("validated"),
      "inv", d.get("invalid"), "nocont", d.get("no_content"), "kern", b.get("tick_kernel_us_avg"),
      "tickwall", b.get("tick_wall_us_avg"), "spt", b.get("streams_per_tick"), "fin", b.get("finalize_items_fused"), b.get("finalize_host"),
      "proxy_cpu", b.get("proxy_cpu_ms_per_1k_req"), "lg_cpu", b.get("loadgen_cpu_ms_per_1k_req"), "rss", b.get("proxy_rss_MB"), "p5ms", b.get("loop_passes_over_5ms"))
EOF
}
bench() {  # name timeout env... -- args...
  local name=$1 to=$2; shift 2
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  timeout -k 10 $to env "${envs[@]}" python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err
  local rc=$?
  summ $name $OUT/$name.json
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -25 $OUT/$name.err; return 1; fi
}
torchrun_bench() {  # name nproc args...
  local name=$1 np=$2; shift 2
  QMX_BENCH_NDEV=${QMX_BENCH_NDEV:-1} timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 500)) bench.py --gpus $np "$@" > $OUT/$name.json 2> $OUT/$name.err
  local rc=$?
  summ $name $OUT/$name.json
  if [ $rc -ne 0 ]; then echo "step $name failed rc=$rc"; tail -30 $OUT/$name.err; return 1; fi
}

for step in "$@"; do
  echo "== $step ($(date +%T))"
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
      tail -3 $OUT/gpu_tests.log ;;
    envtests:*)  # the whole GPU suite under extra env (commas = spaces), e.g. envtests:QMX_PERSISTENT=1
      e=${step#envtests:}; slug=$(echo "$e" | tr -c 'a-zA-Z0-9' '_' | cut -c1-60)
      env ${e//,/ } timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > $OUT/gpu_tests_$slug.log 2>&1 || { echo "gpu tests ($e) failed"; tail -40 $OUT/gpu_tests_$slug.log; exit 1; }
      tail -3 $OUT/gpu_tests_$slug.log ;;
    pytest:*)  # selected GPU test files (commas = spaces), before the full suite
      f=${step#pytest:}; slug=$(echo "$f" | tr -c 'a-zA-Z0-9' '_' | cut -c1-60)
      timeout -k 10 600 python -u -m pytest ${f//,/ } -x -v --timeout 120 --timeout-method thread \
        > $OUT/pytest_$slug.log 2>&1 || { echo "pytest $f failed"; tail -40 $OUT/pytest_$slug.log; exit 1; }
      tail -3 $OUT/pytest_$slug.log ;;
    probe:*)  # a probe binary built on the CPU side (tools/probes/<name>), its JSON lines kept
      pb=${step#probe:}
      timeout -k 10 120 tools/probes/$pb > $OUT/probe_$pb.jsonl 2>&1 || { echo "probe $pb failed"; tail -5 $OUT/probe_$pb.jsonl; exit 1; }
      cat $OUT/probe_$pb.jsonl ;;
    fdprobe)  # which bench-rank step opens a GPU device file
      timeout -k 10 120 python tools/probes/fd_probe.py > $OUT/fdprobe.log 2>&1; cat $OUT/fdprobe.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 \
        || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
      tail -1 $OUT/smoke.log ;;
    bench|bench=*)
      n=${step#bench}; n=${n#=}; n=${n:-1}
      for i in $(seq 1 $n); do bench bench_$i 300 QMX_NOP=1 -- || exit 1; done ;;
    hunt=*)  # N headline runs that go on past an INVALID run (exit 1 with a JSON line saying
             # valid false); the whole body of each invalid response -> invalid_bodies.txt.
             # Any other failure (timeout, crash, no JSON line) ends the session as usual.
      n=${step#hunt=}
      for i in $(seq 1 $n); do
        bench hunt_$i 300 QMX_NOP=1 QMX_LOADGEN_DUMP=$OUT/invalid_bodies.txt -- && continue
        grep -q '"valid": false' $OUT/hunt_$i.json 2>/dev/null || exit 1
        echo "hunt_$i invalid: kept going"
      done ;;
    bench:*)
      a=${step#bench:}; slug=$(echo "$a" | tr -c 'a-zA-Z0-9' '_')
      bench bench_$slug 300 QMX_NOP=1 -- ${a//,/ } || exit 1 ;;
    ab:*)
      rest=${step#ab:}; name=${rest%%:*}; rest=${rest#*:}; envs=${rest%%:*}; a=${rest#*:}
      bench ab_$name 300 ${envs//,/ } -- ${a//,/ } || exit 1 ;;
    scenarios)
      for SC in aggregate4 highqps8 failure paced nonstream1 direct; do
        bench sc_$SC 300 QMX_NOP=1 -- --scenario $SC --steps 10 --warmup 2 $( [ $SC = paced ] || echo --batch 16384 ) || exit 1
      done ;;
    reference)
      bench reference 600 QMX_NOP=1 -- --impl reference --steps 10 --warmup 1 --batch 64 || exit 1 ;;
    refscenarios)  # the upstream proxy on every BASELINE scenario, same harness
      for SC in nonstream1 aggregate4 highqps8 failure; do
        bench ref_$SC 600 QMX_NOP=1 -- --impl reference --scenario $SC --steps 5 --warmup 1 --batch 32 || exit 1
      done ;;
    prof)
      # one-shot launches (tick lanes, QMX_PERSISTENT=0): a persistent grid — the loop-tick grid
      # or a lane's — is one long dispatch, with no per-tick kernel stats
      QMX_TICK_MODE=lanes QMX_PERSISTENT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o native --output-format csv -- \
        python3 bench.py --steps 5 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err \
        || { echo "prof failed"; tail -10 $OUT/bench_prof.err; exit 1; }
      summ prof $OUT/bench_prof.json
      find $OUT/prof -name '*kernel_stats.csv' -exec head -5 {} \; ;;
    pmc:*)
      ctr=${step#pmc:}; slug=$(echo "$ctr" | tr -c 'a-zA-Z0-9' '_' | cut -c1-60)
      QMX_PERSISTENT=0 timeout -s KILL 120 rocprofv3 --pmc ${ctr//,/ } -d $OUT/pmc_$slug -o pmc --output-format csv -- \
        python3 tools/kbench.py --slots 256 --iters 10 > $OUT/pmc_$slug.log 2>&1 \
        || { echo "pmc $ctr failed"; tail -10 $OUT/pmc_$slug.log; exit 1; }
      python3 tools/pmc_summary.py $(find $OUT/pmc_$slug -name '*counter_collection.csv') > $OUT/pmc_$slug.md 2>&1
      grep -v rocclr $OUT/pmc_$slug.md | head -30 ;;
    pmce:*)  # pmce:ENV=V[,ENV=V]:C1,C2 — a one-shot kbench counter pass under extra env
      rest=${step#pmce:}; e=${rest%%:*}; ctr=${rest#*:}
      slug=$(echo "$e:$ctr" | tr -c 'a-zA-Z0-9' '_' | cut -c1-80)
      env ${e//,/ } QMX_PERSISTENT=0 timeout -s KILL 120 rocprofv3 --pmc ${ctr//,/ } -d $OUT/pmce_$slug -o pmc --output-format csv -- \
        python3 tools/kbench.py --slots 256 --iters 10 > $OUT/pmce_$slug.log 2>&1 \
        || { echo "pmce $e $ctr failed"; tail -10 $OUT/pmce_$slug.log; exit 1; }
      python3 tools/pmc_summary.py $(find $OUT/pmce_$slug -name '*counter_collection.csv') > $OUT/pmce_$slug.md 2>&1
      echo "-- $e"; grep -v rocclr $OUT/pmce_$slug.md | grep qmx | head -12 ;;
    pmcgrid:*)  # counters of the production kernel (qmx_tick_persistent: one dispatch, many ticks)
      ctr=${step#pmcgrid:}; slug=$(echo "$ctr" | tr -c 'a-zA-Z0-9' '_' | cut -c1-60)
      timeout -s KILL 120 rocprofv3 --pmc ${ctr//,/ } -d $OUT/pmcg_$slug -o pmc --output-format csv -- \
        python3 tools/kbench.py --grid ${KB_GRID:-16} --slots ${KB_SLOTS:-3} --iters 400 --combos ft > $OUT/pmcg_$slug.log 2>&1 \
        || { echo "pmcgrid $ctr failed"; tail -10 $OUT/pmcg_$slug.log; exit 1; }
      nt=$(python3 -c "
import json
t=0
for l in open('$OUT/pmcg_$slug.log'):
    if l.startswith('{') and 'grid_ticks' in l: t += json.loads(l).get('grid_ticks') or 0
print(int(t))")
      python3 tools/pmc_summary.py --per-tick $nt $(find $OUT/pmcg_$slug -name '*counter_collection.csv') > $OUT/pmcg_$slug.md 2>&1
      grep -v rocclr $OUT/pmcg_$slug.md | head -30 ;;
    kbenchgrid|kbenchgrid:*)  # in-kernel stage split of the production kernel (persistent grid); :ENV=V,... extra env
      e=""; kslug=""
      if [ "$step" != kbenchgrid ]; then e=${step#kbenchgrid:}; kslug=_$(echo "$e" | tr -c 'a-zA-Z0-9' '_' | cut -c1-40); fi
      env ${e//,/ } QMX_STAGE_TIMING=1 timeout -k 10 300 python tools/kbench.py --grid 16 --slots 1,3,22 --iters 100 --combos ft > $OUT/kbenchgrid$kslug.jsonl 2>&1 \
        || { echo "kbenchgrid failed"; tail -5 $OUT/kbenchgrid$kslug.jsonl; exit 1; }
      echo "-- $e"
      grep -v '^{"grid_stats' $OUT/kbenchgrid$kslug.jsonl | python3 -c "
import json, sys
for l in sys.stdin:
    if not l.startswith('{'): continue
    d=json.loads(l); st=d.get('stage_us_per_item',{})
    print(d['slots'], 'wall', d['wall_us_p50'], 'kern', d.get('kernel_us_avg'), 'fence', st.get('stage_fence_us'), [st.get('stage%d_us'%k) for k in range(1,11)])
" ;;
    kbenchshape:*)  # kbenchshape:SHAPE — stage split of the production kernel on another stream shape
      shp=${step#kbenchshape:}
      QMX_STAGE_TIMING=1 timeout -k 10 300 python tools/kbench.py --grid 16 --slots 1,3 --iters 100 --combos ft --shape $shp > $OUT/kbench_$shp.jsonl 2>&1 \
        || { echo "kbenchshape failed"; tail -5 $OUT/kbench_$shp.jsonl; exit 1; }
      grep -v '^{"grid_stats' $OUT/kbench_$shp.jsonl | python3 -c "
import json, sys
for l in sys.stdin:
    if not l.startswith('{'): continue
    d=json.loads(l); st=d.get('stage_us_per_item',{})
    print(d['shape'], d['slots'], 'wall', d['wall_us_p50'], 'kern', d.get('kernel_us_avg'), [st.get('stage%d_us'%k) for k in range(1,11)], {k[6:-3]: v for k, v in st.items() if k.startswith(('stage_s4', 'stage_s6', 'stage_s3'))}, d.get('s3_per_item'))
" ;;
    pmcshape:*)  # pmcshape:SHAPE:C1,C2 — counters of qmx_tick_persistent on another stream shape, per tick
      rest=${step#pmcshape:}; shp=${rest%%:*}; ctr=${rest#*:}; slug=$(echo "${shp}_$ctr" | tr -c 'a-zA-Z0-9' '_' | cut -c1-60)
      timeout -s KILL 120 rocprofv3 --pmc ${ctr//,/ } -d $OUT/pmcs_$slug -o pmc --output-format csv -- \
        python3 tools/kbench.py --grid 16 --slots 3 --iters 400 --combos ft --shape $shp > $OUT/pmcs_$slug.log 2>&1 \
        || { echo "pmcshape $ctr failed"; tail -10 $OUT/pmcs_$slug.log; exit 1; }
      python3 tools/pmc_summary.py --per-tick 400 $(find $OUT/pmcs_$slug -name '*counter_collection.csv') > $OUT/pmcs_$slug.md 2>&1
      grep -v rocclr $OUT/pmcs_$slug.md | head -14 ;;
    kbench)
      QMX_PERSISTENT=0 QMX_STAGE_TIMING=1 timeout -k 10 300 python tools/kbench.py --slots 1,22,64,256 --iters 20 > $OUT/kbench.jsonl 2>&1 \
        || { echo "kbench failed"; tail -5 $OUT/kbench.jsonl; exit 1; }
      python3 -c "
import json
for l in open('$OUT/kbench.jsonl'):
    if not l.startswith('{'): continue
    d=json.loads(l); st=d.get('stage_us_per_item',{})
    print(d.get('filter'),d.get('emit'),d['slots'],d['wall_us_p50'],d['kernel_us_avg'],[st.get('stage%d_us'%k) for k in range(1,11)],
          {k[6:-3]: v for k, v in st.items() if k.startswith('stage_s')}, d.get('s3_per_item', {}))
" ;;
    gpuprocs=*)  # which processes hold the GPU during an N-rank rehearsal (N <= 4 keeps it under the limit)
      n=${step#gpuprocs=}
      python tools/probes/gpu_procs.py $OUT/gpuprocs_$n.txt 60 &
      mon=$!
      QMX_BENCH_FDTRACE=1 torchrun_bench gpuprocs_$n $n --steps 5 --warmup 1 --threads 2 --batch 4096; rc=$?
      grep -A30 "GPU first held" $OUT/gpuprocs_$n.err | head -40
      kill $mon 2>/dev/null; wait $mon 2>/dev/null
      cat $OUT/gpuprocs_$n.txt
      [ $rc -eq 0 ] || exit 1 ;;
    multirank=*)
      n=${step#multirank=}; torchrun_bench multirank_$n $n --steps 5 --warmup 1 --threads 2 --batch 4096 || exit 1 ;;
    selfrank=*)  # bench.py --gpus N launching its own N ranks (no torchrun), sharing GPU 0
      n=${step#selfrank=}
      QMX_BENCH_NDEV=${QMX_BENCH_NDEV:-1} timeout -k 10 400 python bench.py --gpus $n --steps 5 --warmup 1 --threads 2 \
        --batch 4096 > $OUT/selfrank_$n.json 2> $OUT/selfrank_$n.err
      rc=$?; summ selfrank_$n $OUT/selfrank_$n.json
      python3 -c "
import json
d=json.loads([l for l in open('$OUT/selfrank_$n.json') if l.startswith('{')][-1]); s=d.get('spread_check',{})
print('per-rank pids', [r['pid'] for r in d.get('breakdown_per_rank',[])], 'spread', {k: s.get(k) for k in ('ok','requests','invalid','remote_streams','bulk_rounds','mesh_finals','delta_mismatch','worker_nodata','peer_downs','remote_ends','p50_latency_ms','eager_finals','probe_p50_latency_ms','local_probe_p50_latency_ms','hops_us_loaded','hops_us_probe','bulk_formed','rendezvous','finalize_host','remote_texts_gpu','errors')})
for r in s.get('per_rank',[]): print('  ', r)
" || true
      grep "qmx spread\|qmx exchange" $OUT/selfrank_$n.err | head -20
      [ $rc -eq 0 ] || { echo "step selfrank_$n failed rc=$rc"; tail -30 $OUT/selfrank_$n.err; exit 1; } ;;
    selfsc=*)  # selfsc=N:ARGS — bench.py --gpus N (ranks sharing GPU 0) with extra args (commas = spaces)
      rest=${step#selfsc=}; n=${rest%%:*}; a=${rest#*:}; slug=$(echo "$a" | sed -e 's/--scenario,//; s/--steps,[0-9]*,//; s/--warmup,[0-9]*,//; s/--batch,[0-9]*,//' | tr -c 'a-zA-Z0-9' '_' | cut -c1-90)
      QMX_BENCH_NDEV=${QMX_BENCH_NDEV:-1} timeout -k 10 400 python bench.py --gpus $n --threads 2 ${a//,/ } \
        > $OUT/selfsc_${n}_$slug.json 2> $OUT/selfsc_${n}_$slug.err
      rc=$?; summ selfsc_${n}_$slug $OUT/selfsc_${n}_$slug.json
      python3 -c "
import json
d=json.loads([l for l in open('$OUT/selfsc_${n}_$slug.json') if l.startswith('{')][-1])
for r in d.get('breakdown_per_rank',[]): print('  ', r['rank'], r['requests'], 'fin_host', r.get('finalize_host'), r.get('exchange'))
" || true
      [ $rc -eq 0 ] || { echo "step selfsc_$n failed rc=$rc"; tail -30 $OUT/selfsc_${n}_$slug.err; exit 1; } ;;
    spread=*)
      n=${step#spread=}; QMX_XCHG=tcp torchrun_bench spread_$n $n --steps 5 --warmup 1 --threads 2 --batch 4096 --placement spread || exit 1 ;;
    cpuprof)
      bench cpuprof 300 QMX_PROF=$PWD/$OUT/cpu_hip.%p.txt QMX_PROF_US=100 -- --steps 20 --warmup 2 || exit 1
      for f in $OUT/cpu_hip.*.txt; do python3 tools/cpuprof.py $f --top 30 --json $f.json > $f.summary 2>&1 || true; done
      head -30 $OUT/cpu_hip.*.summary ;;
    cpuprofsc:*)  # a scenario with the in-process CPU profiler on the proxy (where its CPU goes)
      SC=${step#cpuprofsc:}
      bench cpuprof_$SC 300 QMX_PROF=$PWD/$OUT/cpu_$SC.%p.txt QMX_PROF_US=100 -- --scenario $SC --steps 10 --warmup 2 \
        --batch 16384 || exit 1
      for f in $OUT/cpu_$SC.*.txt; do python3 tools/cpuprof.py $f --top 40 --json $f.json > $f.summary 2>&1 || true; done
      head -45 $OUT/cpu_$SC.*.summary ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all done"
