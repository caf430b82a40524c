cd $GRAFT_REPO_ROOT
b() { timeout -k 5 250 python bench.py --steps 2 --warmup 1 --cpu-baseline none "$@" 2>gpurun_out/err.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['ms_per_step'],1), d['final_clusters'], r['frac'], round(r['avg_launch_ms']*1e3,1))"; }
for i in 1 2; do echo new c5; b --config c5; echo old c5; KLSH_LIB=$PWD/kmerlsh_amd/lib_ab/libklsh_ab.so b --config c5; done
