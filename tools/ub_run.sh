cd $GRAFT_REPO_ROOT
for e in "X=1" "KLSH_GRID_HINTS=0" "X=2" "KLSH_GRID_HINTS=0"; do
  env $e timeout -k 5 120 python bench.py --steps 3 --warmup 1 --cpu-baseline none 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 $e', round(d['ms_per_step'],1), d['final_clusters'])"
done
env KLSH_GRID_HINTS=0 timeout -k 5 200 python bench.py --config c5 --steps 1 --warmup 1 --cpu-baseline none 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 hints0', round(d['ms_per_step'],1), d['final_clusters'])"
timeout -k 5 200 python bench.py --config c5 --steps 1 --warmup 1 --cpu-baseline none 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 default', round(d['ms_per_step'],1), d['final_clusters'])"
