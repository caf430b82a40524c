#!/bin/bash
# A/B of engine options / library variants on the C2 bench (GPU box).
#   tools/ab.sh ROUNDS "TESTS_K" "name:lib:opts" ...   (lib empty = the default build;
#   TESTS_K empty = no parity tests first)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
rounds=$1; shift
tk=$1; shift
if [ -n "$tk" ]; then
  tools/gpu_steps.sh "abtests:300:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k '$tk'" || exit 1
fi
for round in $(seq 1 "$rounds"); do
  for cfg in "$@"; do
    name=${cfg%%:*}; rest=${cfg#*:}; lib=${rest%%:*}; opt=${rest#*:}
    if [ -n "$lib" ]; then export KLSH_LIB=$lib; else unset KLSH_LIB; fi
    timeout -k 10 200 python bench.py --steps 4 --warmup 1 --cpu-baseline none $opt > gpurun_out/ab/${name}_$round.log 2>&1 || { echo "$name failed"; tail -3 gpurun_out/ab/${name}_$round.log; exit 1; }
    python3 -c "import json,sys; [print('$name $round', round(json.loads(l)['ms_per_step'],1), json.loads(l)['parity'].get('ok'), {k: round(v,1) for k,v in json.loads(l)['phases_ms_per_step'].items() if v}) for l in open('gpurun_out/ab/${name}_$round.log') if l.startswith('{')]"
  done
done
