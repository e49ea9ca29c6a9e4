#!/bin/bash
# round-6 scratch: slice parity, then emulated N = 8 rank and strong configs[4] N = 1 over library variants
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6z}
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/${T}_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for v in ${VARS:-old main}; do
    so=high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib/libhkcsa_$v.so; [ $v = main ] && so=high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib/libhkcsa.so
    HKCSA_LIB=$PWD/$so timeout -k 10 200 python3 tools/shard_emulate.py --nranks 8 --ranks 0 --pos64 > gpurun_out/${T}_e.jsonl 2> gpurun_out/${T}_e.err || { tail -5 gpurun_out/${T}_e.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/${T}_e.jsonl').readline())
print('$v rep $rep emul8', d['build_ms'], {k: v['ms_per_build'] for k,v in d['stages'].items()})"
    HKCSA_LIB=$PWD/$so timeout -k 10 300 python3 -u bench.py --strong --steps 2 --warmup 1 > gpurun_out/${T}_s.json 2> gpurun_out/${T}_s.err || { tail -5 gpurun_out/${T}_s.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/${T}_s.json').read());st=d['detail'].get('stages_ms_total',{})
print('$v rep $rep strong', d['ms_per_step'], {k: round(x['ms']/d['steps'],2) for k,x in st.items() if x['ms']/d['steps'] > 0.5})"
  done
done
