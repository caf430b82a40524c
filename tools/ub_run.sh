cd $GRAFT_REPO_ROOT
b() { timeout -k 5 150 python bench.py --steps 2 --warmup 1 --cpu-baseline none "$@" 2>gpurun_out/err.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['ms_per_step'],1), d['final_clusters'], 'proj frac', r['frac'], r.get('valu'))"; }
for v in pk2 pkst pk2 pkst; do echo $v; KLSH_PROJECT=$v b; done
