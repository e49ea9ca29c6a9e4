#!/bin/bash
# PMC traffic of one bench step (FETCH_SIZE and WRITE_SIZE in separate passes, kernel trace only).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$c -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --patterns 0 > gpurun_out/pmc_$c.json 2> gpurun_out/pmc_$c.err
  rc=$?
  echo "$c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
ls -R gpurun_out/pmc_FETCH_SIZE | head
