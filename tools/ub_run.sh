cd $GRAFT_REPO_ROOT
b() { timeout -k 5 200 python bench.py --steps 2 --warmup 1 --cpu-baseline none "$@" 2>gpurun_out/err.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],1), d['final_clusters'])"; }
for i in 1 2; do echo new c2; b; echo old c2; KLSH_LIB=$PWD/kmerlsh_amd/lib_ab/libklsh_ab.so b; done
echo new c4; b --config c4
echo old c4; KLSH_LIB=$PWD/kmerlsh_amd/lib_ab/libklsh_ab.so b --config c4
