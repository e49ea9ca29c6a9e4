set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_dropin.py --durations=3 -m gpu > gpurun_out/ab_tests.log 2>&1 &&
TAG=r5z STEPS="profen" bash tools/gpu_suite.sh
