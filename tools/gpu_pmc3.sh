#!/bin/bash
# SQ counters of the slice kernels only (emulated N=8 rank 0), two --pmc passes; summary printed.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${TAG:-p3}
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "${KRE:-k_slice}" --output-format csv \
      -d gpurun_out/${tag}_$i -o run -- ${CMD:-python3 tools/shard_emulate.py --nranks 8 --ranks 0 --reps 1} > gpurun_out/${tag}_$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/${tag}_$i.log; exit 1; }
done
python3 tools/pmc_sq_summary.py gpurun_out $tag
