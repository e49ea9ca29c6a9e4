#!/bin/bash
# Round-3 measurement: the default bench line (all legs), a bucket-sort phase trace, the sharded and
# strong N=1 lines, then a rocprofv3 kernel-stats pass over a short default bench.  Each GPU step has its
# own time limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3c
export TMPDIR=/tmp
O=gpurun_out/r3c
step() {   # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$O/$name.err"; tail -c 600 "$O/$name.out"; echo
  [ $rc -eq 0 ] || exit $rc
}
step bench 400 python3 bench.py
step trace 200 env HKCSA_BS_TRACE=1 python3 bench.py --steps 1 --warmup 0 --patterns 0 --no-cpu-baseline --no-legs --no-eps --no-pcie
grep -h "trace\]" "$O/trace.err"
[ -n "$SKIP_SHARD" ] || step sharded 300 python3 bench.py --sharded --steps 5 --warmup 1 --no-cpu-baseline --no-legs --no-eps --no-pcie
[ -n "$SKIP_SHARD" ] || step strong 400 python3 bench.py --strong --steps 3 --warmup 1 --no-cpu-baseline --no-legs --no-eps --no-pcie
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-pcie > "$GRAFT_REPO_ROOT/$O/prof.out" 2> "$GRAFT_REPO_ROOT/$O/prof.err"
rc=$?; echo "== rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$GRAFT_REPO_ROOT/$O/prof.err"; exit $rc; }
find "$GRAFT_REPO_ROOT/$O/prof" -name "*kernel_stats.csv" | head -3
exit 0
