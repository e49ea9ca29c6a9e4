#!/bin/bash
# WT A/B: the WT / query parity tests, then the bench (with the sigma = 256 and printable legs) with
# an env toggle (AB_VAR) on / off, printing the WT build and the partition kernel's launch time.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
( while sleep 60; do date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 200 --timeout-method thread -k "${K:-wt or count or locate or rank or occ or golden}" > gpurun_out/wt_tests.log 2>&1 || { tail -30 gpurun_out/wt_tests.log; exit 1; }
tail -2 gpurun_out/wt_tests.log
for v in ${AB_VALS:-1 0 1 0}; do
  env $AB_VAR=$v timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-eps --no-pcie > gpurun_out/wtab_$v.json 2> gpurun_out/wtab_$v.err || { tail -5 gpurun_out/wtab_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/wtab_$v.json').read().strip().splitlines()[-1]); de=d['detail']; l=de['legs']['sigma256']
print('$AB_VAR=$v', 'dna wt', de['wt_build_ms'], 'part', de['wt_roofline']['avg_launch_ms'], de['wt_roofline']['frac'], '| s256 wt', l['wt_build_ms'], 'part', l['wt_roofline']['avg_launch_ms'], l['wt_roofline']['frac'], '| locate', de['locate']['locate_patterns_per_s'])"
done
