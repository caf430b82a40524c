#!/bin/bash
# Round profiles on the GPU box (run through gpurun from the repo root):
#   C2 bench line, rocprofv3 kernel stats + trace of one C2 step, FETCH_SIZE / WRITE_SIZE of the
#   kernel classes (projection, sort, runs + k_tail_local, small-run screen, small-run merge,
#   k_merge_tail, compaction; separate --pmc passes, the engine printing a progress line every 25
#   iterations), kernel stats of C4 and C5.  Outputs under gpurun_out/prof/; then
#   python tools/pmc_summary.py <tag> && python tools/check_rooflines.py <tag>
#   tools/collect_profiles.sh [c2|pmc|c45|all] | pmcx [c2] [c4] [c5]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/prof
mkdir -p $out
set -o pipefail
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
B="python bench.py --steps 1 --warmup 0 --cpu-baseline none --option progress=25"
if [ "$1" != pmc ] && [ "$1" != c45 ]; then
  run c2_bench 300 python bench.py --steps 3 --warmup 1
  run c2_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c2_stats -o run -- $B
fi
if [ "$1" = pmc ] || [ "$1" = all ]; then
  # class:regex (tools/pmc_summary.py's CLASSES); every pass also collects k_project, whose second
  # dispatch marks the main loop's start
  for spec in "project:k_project" "screen:k_small_screen" "small:k_merge_small" "sort:k_sort_" \
              "tail:k_merge_tail" "runs:k_runs_|k_tail_local" "compact:k_compact"; do
    c=${spec%%:*}; rx="${spec#*:}|k_project"
    run c2_fetch_$c 300 rocprofv3 --pmc FETCH_SIZE --output-format csv --kernel-include-regex "$rx" -d $out/c2_fetch_$c -o run -- $B
    run c2_write_$c 300 rocprofv3 --pmc WRITE_SIZE --output-format csv --kernel-include-regex "$rx" -d $out/c2_write_$c -o run -- $B
  done
fi
# counter passes of the merge classes (C2's k_merge_big classes) and of C4 / C5's headline classes:
#   pmcx [c2] [c4] [c5]  (one FETCH_SIZE and one WRITE_SIZE pass per class)
pmc_pass() {  # cfg class regex bench-args...
  local cfg=$1 c=$2 rx="$3|k_project"; shift 3
  run ${cfg}_fetch_$c 400 rocprofv3 --pmc FETCH_SIZE --output-format csv --kernel-include-regex "$rx" -d $out/${cfg}_fetch_$c -o run -- "$@"
  run ${cfg}_write_$c 400 rocprofv3 --pmc WRITE_SIZE --output-format csv --kernel-include-regex "$rx" -d $out/${cfg}_write_$c -o run -- "$@"
}
if [ "$1" = pmcx ]; then
  shift
  for cfg in "$@"; do
    case $cfg in
      c2)
        for c in 128 192 384 896; do pmc_pass c2 big$c "k_merge_big<64, $c," $B; done ;;
      c4)
        B4="python bench.py --config c4 --steps 1 --warmup 0 --cpu-baseline none --option progress=25"
        pmc_pass c4 big384 "k_merge_big<32, 384," $B4
        pmc_pass c4 huge "k_merge_long" $B4 ;;
      c5)
        B5="python bench.py --config c5 --steps 1 --warmup 0 --cpu-baseline none --option progress=25"
        pmc_pass c5 project "k_project_mfma_wide|k_project_fix" $B5
        pmc_pass c5 small "k_merge_group_wide" $B5
        pmc_pass c5 big384 "k_merge_big_wide<384" $B5 ;;
    esac
  done
  exit 0
fi
if [ "$1" = all ] || [ "$1" = c45 ]; then
  run c4_bench 400 python bench.py --config c4 --steps 2 --warmup 1 --cpu-baseline none
  run c5_bench 400 python bench.py --config c5 --steps 2 --warmup 1 --cpu-baseline none
  run c4_stats 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c4_stats -o run -- python bench.py --config c4 --steps 1 --warmup 0 --cpu-baseline none
  run c5_stats 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/c5_stats -o run -- python bench.py --config c5 --steps 1 --warmup 0 --cpu-baseline none
fi
exit 0
