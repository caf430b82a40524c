cd $GRAFT_REPO_ROOT
export KLSH_MERGE_PROF=1
KLSH_LIB=$PWD/kmerlsh_amd/lib_ab/libklsh_prof.so timeout -k 5 120 python bench.py --steps 1 --warmup 0 --iterations 1 --cpu-baseline none 2>&1 | grep -E "prof|timed"
KLSH_LIB=$PWD/kmerlsh_amd/lib_ab/libklsh_prof.so timeout -k 5 120 python bench.py --steps 1 --warmup 0 --cpu-baseline none 2>&1 | grep -E "prof|timed"
