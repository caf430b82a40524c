cd $GRAFT_REPO_ROOT
for e in "X=1" "KLSH_PROJECT=pk2"; do
  env $e timeout -k 5 200 python bench.py --config c5 --steps 1 --warmup 1 --cpu-baseline none 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$e', round(d['ms_per_step'],1), d['final_clusters'], 'proj ms', round(d['phases_ms_per_step']['project'],1), 'avg launch us', round(r['avg_launch_ms']*1e3,1), 'frac', r['frac'])"
done
