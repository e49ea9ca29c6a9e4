#!/bin/bash
# SQ counters of the slice kernels (emulated N=8 rank 0) and of the single-GPU build kernels (1 GiB
# sigma=4 step), two --pmc passes each; summaries printed per kernel.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # tag regex cmd...
  tag=$1; re=$2; shift 2
  i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "$re" --output-format csv \
        -d gpurun_out/p2_${tag}_$i -o run -- "$@" > gpurun_out/p2_${tag}_$i.log 2>&1 || { echo "$tag pass $i rc=$?"; tail -5 gpurun_out/p2_${tag}_$i.log; exit 1; }
  done
}
run slice "k_slice" python3 tools/shard_emulate.py --nranks 8 --ranks 0 --reps 1 && \
run build "bucket_sort_fast|k_cpart|wt_partition|k_bucket_hist" python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --patterns 0 --wt-reps 1 --leg-steps 1 && \
python3 tools/pmc_sq_summary.py gpurun_out p2_slice p2_build
