#!/bin/bash
# Round-2 profile: kernel-trace stats of the default bench, HBM traffic (FETCH_SIZE / WRITE_SIZE in
# separate passes), SQ issue / LDS counters of the bucket sort and radix passes, L2 hit + occupancy of
# the batched count kernel.  Every pass runs the program directly after `--`.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r2}
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_stats -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_stats.json 2> gpurun_out/${TAG}_stats.err \
  || { echo "stats rc=$?"; tail -5 gpurun_out/${TAG}_stats.err; exit 1; }
echo stats ok
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_pmc_$c -o run -- $B \
      > gpurun_out/${TAG}_pmc_$c.json 2> gpurun_out/${TAG}_pmc_$c.err || { echo "$c rc=$?"; tail -5 gpurun_out/${TAG}_pmc_$c.err; exit 1; }
  echo "$c ok"
done
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex "k_synth|bucket_sort|onesweep|cpart|bucket_hist|byte_hist|wt_" --output-format csv \
      -d gpurun_out/${TAG}_sq_$i -o run -- $B > gpurun_out/${TAG}_sq_$i.log 2>&1 || { echo "sq $i rc=$?"; tail -5 gpurun_out/${TAG}_sq_$i.log; exit 1; }
  echo "sq set $i ok"
done
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-include-regex "k_synth|k_count" --output-format csv -d gpurun_out/${TAG}_count -o run -- $B \
    > gpurun_out/${TAG}_count.log 2>&1 || { echo "count rc=$?"; tail -5 gpurun_out/${TAG}_count.log; exit 1; }
echo "count pmc ok"
