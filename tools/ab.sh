#!/bin/bash
# A/B of engine builds / environment settings on the GPU box, interleaved: one bench line per
# setting per round.  tools/ab.sh ROUNDS "ENV=.. ENV2=.." "..." ...   ("" = the product build)
# Extra bench flags: AB_ARGS (default: --steps 5 --warmup 1 --cpu-baseline none).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
rounds=$1; shift
args=${AB_ARGS:---steps 5 --warmup 1 --cpu-baseline none}
for r in $(seq 1 "$rounds"); do
  i=0
  for cfg in "$@"; do
    i=$((i + 1))
    log=gpurun_out/ab/r${r}_$i.log
    env $cfg timeout -k 10 300 python -u bench.py $args > $log 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "[$i] $cfg rc=$rc"; tail -5 $log; exit $rc; }
    python - "$log" "$i" "$cfg" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
ks = d["roofline"].get("kernels", [])
top = " ".join(f"{k['class']}={k['ms_per_step']:.1f}" for k in ks[:7])
print(f"[{sys.argv[2]}] {sys.argv[3][:44]:44s} {d['ms_per_step']:8.2f} ms parity={d['parity'].get('ok')} | {top}", flush=True)
PY
  done
done
