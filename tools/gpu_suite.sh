#!/bin/bash
# One gpurun call's worth of evidence on the current tree.  usage (on the box):
#   TAG=r5a STEPS="tests smoke bench prof emul8 strong gap" bash tools/gpu_suite.sh
# Steps (each under its own time limit, the call stops at the first failure):
#   tests   the whole -m gpu suite (config tests first, multi-process tests last; conftest.py)
#   smoke   __graft_entry__.smoke()
#   bench   the default bench line (all legs)            -> gpurun_out/<TAG>_bench.json
#   prof    tools/kprof.py on a 1-step bench of the 1 GiB sigma=4 build (stats, HBM traffic, SQ counters,
#           one row per demangled kernel)                 -> gpurun_out/kprof_<TAG>.json
#   profen  the same on the English-like 200 MiB leg     -> gpurun_out/kprof_<TAG>en.json
#   strong  the strong configs[4] line at N = 1           -> gpurun_out/<TAG>_strong.json
#   emul8   emulated N = 8 rank 0 / 7                     -> gpurun_out/<TAG>_emul8.jsonl
#   profemul8 / profstrong   tools/kprof.py on one emulated N = 8 rank / one strong 4 GiB step
#   gap     one-step kernel trace with host gaps          -> gpurun_out/<TAG>_gap.txt
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r5}
mkdir -p gpurun_out
B1="python3 bench.py --steps 1 --warmup 0 --no-legs --no-cpu-baseline --no-pcie --no-harness --no-eps --patterns 0"
for s in ${STEPS:-tests smoke bench}; do
  echo "== $s $(date +%T)"
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest -x -v --durations=40 --timeout 600 --timeout-method thread -m gpu tests \
        > gpurun_out/${TAG}_gpu_tests.log 2>&1
      rc=$?; tail -4 gpurun_out/${TAG}_gpu_tests.log ;;
    quick)
      timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests} \
        > gpurun_out/${TAG}_gpu_quick.log 2>&1
      rc=$?; tail -4 gpurun_out/${TAG}_gpu_quick.log ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
      rc=$?; cat gpurun_out/${TAG}_smoke.log ;;
    bench)
      timeout -k 10 600 python3 -u bench.py ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
      rc=$?; tail -6 gpurun_out/${TAG}_bench.err; cut -c1-400 gpurun_out/${TAG}_bench.json ;;
    prof)
      timeout -k 10 900 python3 tools/kprof.py --tag ${TAG} -- $B1 > gpurun_out/${TAG}_kprof.log 2>&1
      rc=$?; head -12 gpurun_out/${TAG}_kprof.log | cut -c1-300 ;;
    profen)
      timeout -k 10 900 python3 tools/kprof.py --tag ${TAG}en -- python3 bench.py --only-leg english --leg-steps 1 --patterns 1000 --wt-reps 1 --query-reps 1 \
        > gpurun_out/${TAG}en_kprof.log 2>&1
      rc=$?; head -12 gpurun_out/${TAG}en_kprof.log | cut -c1-300 ;;
    profemul8)
      timeout -k 10 900 python3 tools/kprof.py --tag ${TAG}e8 -- python3 tools/shard_emulate.py --nranks 8 --ranks 0 --pos64 --reps 1 \
        > gpurun_out/${TAG}e8_kprof.log 2>&1
      rc=$?; head -12 gpurun_out/${TAG}e8_kprof.log | cut -c1-300 ;;
    profstrong)
      timeout -k 10 900 python3 tools/kprof.py --tag ${TAG}st -- python3 bench.py --strong --steps 1 --warmup 0 \
        > gpurun_out/${TAG}st_kprof.log 2>&1
      rc=$?; head -12 gpurun_out/${TAG}st_kprof.log | cut -c1-300 ;;
    strong)
      timeout -k 10 300 python3 -u bench.py --strong --steps 3 --warmup 1 > gpurun_out/${TAG}_strong.json 2> gpurun_out/${TAG}_strong.err
      rc=$?; cut -c1-300 gpurun_out/${TAG}_strong.json ;;
    emul8)
      timeout -k 10 300 python3 tools/shard_emulate.py --nranks 8 --ranks 0 7 --pos64 > gpurun_out/${TAG}_emul8.jsonl 2> gpurun_out/${TAG}_emul8.err
      rc=$?; cut -c1-200 gpurun_out/${TAG}_emul8.jsonl ;;
    gap)
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_gap -o run -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --patterns 0 --no-legs --no-pcie --no-eps --no-harness \
        > gpurun_out/${TAG}_gap.json 2> gpurun_out/${TAG}_gap.err
      rc=$?
      [ $rc -eq 0 ] && python3 tools/gap_trace.py gpurun_out/${TAG}_gap/run_kernel_trace.csv > gpurun_out/${TAG}_gap.txt && tail -2 gpurun_out/${TAG}_gap.txt ;;
    *) echo "unknown step $s"; rc=2 ;;
  esac
  [ $rc -eq 0 ] || { echo "step $s failed rc=$rc"; exit $rc; }
done
echo "== done $(date +%T)"
