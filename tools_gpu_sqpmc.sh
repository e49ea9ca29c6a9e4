#!/bin/bash
# SQ counters (issue / wait / LDS) of the text-scanning kernels, one rocprofv3 --pmc pass each set.
# usage: bash tools_gpu_sqpmc.sh   (env PER_RANK, NRANKS)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
PER=${PER_RANK:-134217728}
NR=${NRANKS:-8}
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "pack_select|pack_keys|shard_hist" --output-format csv \
      -d gpurun_out/sqpmc_$i -o run -- python3 tools_shard_emulate.py --per-rank $PER --nranks $NR --ranks 0 --reps 1 \
      > gpurun_out/sqpmc_$i.log 2>&1
  rc=$?
  echo "set $i rc=$rc"; tail -2 gpurun_out/sqpmc_$i.log
  [ $rc -eq 0 ] || exit $rc
done
