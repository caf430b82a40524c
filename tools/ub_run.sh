cd $GRAFT_REPO_ROOT
for nb in "9469536 23" "4000000 22" "2000000 21"; do
  set -- $nb
  timeout -k 5 60 ./tools/ubench_sort $1 $2 30 || exit 1
  KLSH_SORT_BIGTILE=1 timeout -k 5 60 ./tools/ubench_sort $1 $2 30 || exit 1
done
