cd $GRAFT_REPO_ROOT
for e in "X=1" "KLSH_LIB=$PWD/kmerlsh_amd/lib_ab/libklsh_ab.so" "X=2" "KLSH_LIB=$PWD/kmerlsh_amd/lib_ab/libklsh_ab.so"; do
  env $e timeout -k 5 120 python bench.py --steps 3 --warmup 1 --cpu-baseline none 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('${e:0:20}', round(d['ms_per_step'],1), d['final_clusters'])"
done
