#!/bin/bash
# A/B of the bucket-sort fast path (HKCSA_BS_FAST=1 vs 0) on the 1 GiB sigma=4 bench step, then the
# phase stamps of both kernels (HKCSA_BS_TRACE=1).  TESTS=1 runs the GPU suite first.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -40 gpurun_out/gputest.log; exit 1; }
  tail -2 gpurun_out/gputest.log
fi
for f in 1 0; do
HKCSA_BS_FAST=$f timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-legs --no-cpu-baseline ${BARGS} > gpurun_out/ab_$f.json 2> gpurun_out/ab_$f.err || { tail gpurun_out/ab_$f.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/ab_$f.json'));r=d['roofline'];print('fast=$f', d['ms_per_step'], r['kernel'], r['avg_launch_ms'], [(o['kernel'],o['avg_launch_ms']) for o in r['others']], d['detail']['build_info'][:10])"
HKCSA_BS_TRACE=1 HKCSA_BS_FAST=$f timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-legs --no-cpu-baseline --patterns 0 ${BARGS} 2>&1 >/dev/null | grep trace
done
