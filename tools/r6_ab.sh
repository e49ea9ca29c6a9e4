#!/bin/bash
# round-6 scratch: parity of the bucket path, then A/B of the bucket sort variants
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6a}
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/${T}_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
fi
B="python bench.py --steps ${STEPS:-20} --warmup 5 --no-legs --no-cpu-baseline --no-eps --no-pcie --no-harness --patterns 0"
for rep in 1 2; do
  for v in ${VARS:-base main main:HKCSA_BS_PERSIST=0}; do
    lib=${v%%:*}; envs=""; [ "$lib" != "$v" ] && envs=${v#*:}; envs=${envs//,/ }
    so=high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib/libhkcsa_$lib.so; [ $lib = main ] && so=high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib/libhkcsa.so
    env $envs HKCSA_LIB=$PWD/$so timeout -k 10 100 $B > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err || { tail -5 gpurun_out/${T}_ab.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/${T}_ab.json').read());st=d['detail']['stages_ms_total']
print('$v rep $rep', d['ms_per_step'], d['roofline']['frac'], {k: round(v['ms']/d['steps'],3) for k,v in st.items() if v['ms']/d['steps'] > 0.2})"
  done
done
for v in ${TRACES:-HKCSA_X=1 HKCSA_BS_PERSIST=0}; do
  env ${v//,/ } HKCSA_BS_TRACE=1 timeout -k 10 100 python bench.py --steps 1 --warmup 1 --no-legs --no-cpu-baseline --no-eps --no-pcie --no-harness --patterns 0 2>&1 >/dev/null | grep 'bucket_sort trace' | tail -1 | sed "s/^/$v /"
done
