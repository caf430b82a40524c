#!/bin/bash
# PMC passes over the small-run merge and the round-3 fp16 screen (one counter group per run).
#   tools/pmc_small_screen.sh <lib> <outdir> [env...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
lib=$1; out=$2; shift 2
mkdir -p "$out"
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
            "SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS FETCH_SIZE"; do
  i=$((i + 1))
  echo "=== pass $i: $ctrs"
  env "$@" KLSH_LIB="$lib" timeout -s KILL 240 rocprofv3 --pmc $ctrs --output-format csv \
      --kernel-include-regex "k_small_screen|k_merge_small" -d "$out/p$i" -o run -- python3 tools/run_c2.py \
      > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$out/p$i.log"; exit 1; }
  tail -1 "$out/p$i.log"
done
