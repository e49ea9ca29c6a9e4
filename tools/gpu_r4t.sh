#!/bin/bash
# Round 4 diagnostics: phase stamps of the slice pass A (HKCSA_SL_TRACE) at emulated N = 2 / 8 and of the
# LDS bucket sort (HKCSA_BS_TRACE) on the 1 GiB step, final library.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
HKCSA_SL_TRACE=1 timeout -k 10 300 python3 tools/shard_emulate.py --nranks 2 --ranks 0 > gpurun_out/r4t_sl2.jsonl 2> gpurun_out/r4t_sl2.err || exit $?
grep "trace\]" gpurun_out/r4t_sl2.err | head -3
HKCSA_SL_TRACE=1 timeout -k 10 300 python3 tools/shard_emulate.py --nranks 8 --ranks 0 > gpurun_out/r4t_sl8.jsonl 2> gpurun_out/r4t_sl8.err || exit $?
grep "trace\]" gpurun_out/r4t_sl8.err | head -3
HKCSA_BS_TRACE=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-legs --no-cpu-baseline --no-pcie \
  --no-harness --no-eps --patterns 0 > gpurun_out/r4t_bs.json 2> gpurun_out/r4t_bs.err || exit $?
grep "trace\]" gpurun_out/r4t_bs.err | head -3
