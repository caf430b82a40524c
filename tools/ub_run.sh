cd $GRAFT_REPO_ROOT
b() { timeout -k 5 200 python bench.py --steps 2 --warmup 1 --cpu-baseline none "$@" 2>gpurun_out/err.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],1), d['final_clusters'])"; }
echo c4; b --config c4
echo c2; b
echo c2; b
