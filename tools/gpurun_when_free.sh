#!/bin/bash
# Host-side helper: run one gpurun call, re-submitting it only while the pool reports no free box or
# slot (exit code 3: nothing ran, nothing charged); any other outcome ends it.  usage:
#   tools/gpurun_when_free.sh OUT TIMEOUT CMD...
out=$1; to=$2; shift 2
for try in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$out" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 60
done
exit 3
