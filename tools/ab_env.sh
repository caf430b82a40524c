#!/bin/bash
# A/B of engine environment switches on the GPU box: one C2 bench line per setting.
#   tools/ab_env.sh "NAME=VAL NAME2=VAL" "..." ...   (an empty string = the default build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
i=0
for cfg in "$@"; do
  i=$((i + 1))
  echo "=== [$i] $cfg"
  env $cfg timeout -k 10 180 python -u bench.py --steps ${AB_STEPS:-5} --warmup 1 --cpu-baseline none > gpurun_out/ab/$i.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/ab/$i.log; exit $rc; }
  python - "$i" "$cfg" <<'PY'
import json, sys
line = [l for l in open("gpurun_out/ab/%s.log" % sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print("[%s] %-50s %8.2f ms  parity %s  small %.1f ms" % (sys.argv[1], sys.argv[2], d["ms_per_step"], d["parity"]["ok"], d["phases_ms_per_step"]["small"]))
PY
done
