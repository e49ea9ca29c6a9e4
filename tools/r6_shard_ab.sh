cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6o}
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_slices.py tests/test_gpu_dist.py} > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/shard_emulate.py --nranks 8 --ranks 0 --pos64 > gpurun_out/${T}_emul8.jsonl 2> gpurun_out/${T}_emul8.err || exit 1
cut -c1-420 gpurun_out/${T}_emul8.jsonl
HKCSA_SL_TRACE=1 timeout -k 10 300 python3 tools/shard_emulate.py --nranks 8 --ranks 0 --pos64 --reps 1 2>&1 >/dev/null | grep trace | head -2
B="python bench.py --steps 20 --warmup 5 --no-legs --no-cpu-baseline --no-eps --no-pcie --no-harness --patterns 0"
timeout -k 10 100 $B > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err || exit 1
python3 -c "
import json;d=json.loads(open('gpurun_out/${T}_ab.json').read());st=d['detail']['stages_ms_total']
print('headline', d['ms_per_step'], d['roofline']['frac'], {k: round(v['ms']/d['steps'],3) for k,v in st.items() if v['ms']/d['steps'] > 0.2})"
