#!/bin/bash
# round-6 scratch: emulated N = 8 rank 0 stage times, A/B over library variants (VARS: names; main = libhkcsa.so)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6e}
for rep in 1 2; do
  for v in ${VARS:-main}; do
    so=high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib/libhkcsa_$v.so; [ $v = main ] && so=high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib/libhkcsa.so
    HKCSA_LIB=$PWD/$so timeout -k 10 200 python3 tools/shard_emulate.py --nranks ${NR:-8} --ranks 0 --pos64 ${EXTRA} > gpurun_out/${T}_e.jsonl 2> gpurun_out/${T}_e.err || { tail -5 gpurun_out/${T}_e.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/${T}_e.jsonl').readline())
print('$v rep $rep', d['build_ms'], {k: v['ms_per_build'] for k,v in d['stages'].items()})"
  done
done
