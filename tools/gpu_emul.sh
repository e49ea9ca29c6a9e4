#!/bin/bash
# Emulated per-rank sharded builds on one GPU (EMUL_ARGS lines, ';'-separated), with slice diagnostics.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export HKCSA_SHARD_DEBUG=1
IFS=';' read -ra RUNS <<< "${EMUL_ARGS:---nranks 8 --ranks 0 3 --pos64}"
i=0
for a in "${RUNS[@]}"; do
  timeout -k 10 300 python3 tools/shard_emulate.py $a > gpurun_out/emul_$i.jsonl 2> gpurun_out/emul_$i.err
  rc=$?; echo "== $a rc=$rc"; grep -E "^\[(shard|slice)\]" gpurun_out/emul_$i.err | head -8; cat gpurun_out/emul_$i.jsonl
  [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
