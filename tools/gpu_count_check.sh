cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread -k "oracle or golden or dropin or csa or sampled" > gpurun_out/t9.log 2>&1 || { tail -30 gpurun_out/t9.log; exit 1; }
tail -2 gpurun_out/t9.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/p9 -o run -- python3 bench.py --steps 2 --warmup 1 --no-legs --no-cpu-baseline --no-pcie > gpurun_out/b9.json 2> gpurun_out/b9.err || { tail -5 gpurun_out/b9.err; exit 1; }
cat gpurun_out/b9.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['locate_patterns_per_s'], d['detail']['wt_build_ms'])"
