#!/bin/bash
# Round 4: parity on the reverted sort + half-staged pass B + locate/refinement changes, A/B base vs main,
# bucket-sort write traffic with the BWT or SA stores removed (diagnostic libraries), the 4 GiB tests.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_bucket.py tests/test_gpu_slices.py tests/test_gpu_dropin.py 2>&1 | tee gpurun_out/r4f_quick.log
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
LIBS="base main" REPS="1 2" bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r4f_ab.log
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
L=$PWD/high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib
for v in main nobwt nosa; do
  lib=$L/libhkcsa_$v.so; [ "$v" = main ] && lib=$L/libhkcsa.so
  HKCSA_LIB=$lib timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex bucket_sort_fast --output-format csv \
      -d gpurun_out/r4f_w_$v -o run -- python3 bench.py --steps 1 --warmup 0 --no-legs --no-cpu-baseline --no-pcie \
      --no-harness --no-eps --patterns 0 > gpurun_out/r4f_w_$v.json 2> gpurun_out/r4f_w_$v.err
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, glob
for v in ("main", "nobwt", "nosa"):
    for f in glob.glob(f"gpurun_out/r4f_w_{v}/**/run_counter_collection.csv", recursive=True):
        rows = [r for r in csv.DictReader(open(f))]
        big = max(int(r["Grid_Size"]) for r in rows)
        vals = [float(r["Counter_Value"]) for r in rows if int(r["Grid_Size"]) == big]
        print(v, "WRITE_SIZE GB per launch", [round(x * 1024 / 1e9, 3) for x in vals])
PY
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_scale.py 2>&1 | tee gpurun_out/r4f_scale.log
exit ${PIPESTATUS[0]}
