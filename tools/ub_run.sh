cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
b() { timeout -k 5 150 python bench.py --steps 2 --warmup 1 --cpu-baseline none "$@" 2>gpurun_out/err.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],1), d['final_clusters'])"; }
echo shard1-all; KLSH_SHARD_MIN_ROWS=0 b --shard1
KLSH_SHARD_MIN_ROWS=0 timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sh1 -o run -- python bench.py --steps 1 --warmup 0 --cpu-baseline none --shard1 > gpurun_out/sh1.log 2>&1 || exit 1
f=$(find gpurun_out/sh1 -name '*kernel_trace.csv' | head -1)
python tools/trace_iter.py $f 0,150 | grep -E "iteration|part|bin_|unpack"
