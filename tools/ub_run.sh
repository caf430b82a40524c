cd $GRAFT_REPO_ROOT
for v in "" lsd; do
KLSH_SORT=$v KLSH_ITER_LOG=gpurun_out/iter_$v.log timeout -k 5 120 python bench.py --steps 1 --warmup 1 --cpu-baseline none > gpurun_out/b_$v.log 2>&1 || exit 1
tail -1 gpurun_out/b_$v.log | cut -c 1-300
done
