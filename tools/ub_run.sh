cd $GRAFT_REPO_ROOT
for nb in "390000 18" "1500000 20" "700000 19" "150000 17"; do
 for sv in "" "0"; do
   KLSH_SORT_WIDE=$sv timeout -k 5 30 tools/ubench_sort $nb 20 || exit 1
 done
done
for e in "X=1" "KLSH_SORT_WIDE=0" "X=2"; do
  env $e timeout -k 5 120 python bench.py --steps 3 --warmup 1 --cpu-baseline none 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$e', round(d['ms_per_step'],1), d['final_clusters'])"
done
