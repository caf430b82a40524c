cd $GRAFT_REPO_ROOT
for e in "X=1" "KLSH_QUEUE_AHEAD=0" "X=2" "KLSH_QUEUE_AHEAD=0"; do
  env $e timeout -k 5 120 python bench.py --steps 3 --warmup 1 --cpu-baseline none 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$e', round(d['ms_per_step'],1), d['final_clusters'], round(r['avg_launch_ms']*1e3,1))"
done
