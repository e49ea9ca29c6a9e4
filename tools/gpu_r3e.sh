cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
HKCSA_SL_TRACE=1 timeout -k 10 200 python3 tools/shard_emulate.py --nranks 8 --ranks 0 --reps 1 --pos64 > gpurun_out/tr8.json 2> gpurun_out/tr8.err || { tail gpurun_out/tr8.err; exit 1; }
grep "trace\]" gpurun_out/tr8.err | tail -2
EMUL_ARGS="--nranks 2 --ranks 0 1;--nranks 4 --ranks 0 --pos64;--nranks 8 --ranks 0 7 --pos64" bash tools/gpu_emul.sh
