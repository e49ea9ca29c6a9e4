#!/bin/bash
# Final round-3 evidence: emulated per-rank sharded builds (N = 2 / 4 / 8) and the SQ counters of the
# bucket sort and the partition passes on the final tree.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
EMUL_ARGS="--nranks 2 --ranks 0 1;--nranks 4 --ranks 0 --pos64;--nranks 8 --ranks 0 7 --pos64" bash tools/gpu_emul.sh || exit 1
KRE="bucket_sort_fast|cpart|slice_cpart|slice_hist" bash tools/gpu_sqpmc.sh > gpurun_out/sq_final.txt 2>&1 || { tail -20 gpurun_out/sq_final.txt; exit 1; }
python3 tools/pmc_sq_summary.py gpurun_out sqpmc > gpurun_out/sq_final.json && head -c 1500 gpurun_out/sq_final.json
