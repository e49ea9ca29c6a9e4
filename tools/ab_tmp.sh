set -o pipefail
V=high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib/libhkcsa_w1024.so
L="python3 bench.py --only-leg english --leg-steps 3 --patterns 1000 --wt-reps 1 --query-reps 1"
P="python3 bench.py --only-leg protein --leg-steps 2 --patterns 1000 --wt-reps 1 --query-reps 1"
HKCSA_LIB=$V timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_english.py tests/test_gpu_slices.py -m gpu > gpurun_out/ab_tests.log 2>&1 &&
for i in 1 2; do
  timeout -k 10 200 $L > gpurun_out/ab_wA_$i.json 2> gpurun_out/ab_wA_$i.err &&
  HKCSA_LIB=$V timeout -k 10 200 $L > gpurun_out/ab_wB_$i.json 2> gpurun_out/ab_wB_$i.err || exit 1
done &&
timeout -k 10 200 $P > gpurun_out/ab_wpA.json 2> gpurun_out/ab_wpA.err &&
HKCSA_LIB=$V timeout -k 10 200 $P > gpurun_out/ab_wpB.json 2> gpurun_out/ab_wpB.err
