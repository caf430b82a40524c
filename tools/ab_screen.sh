#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
tools/gpu_steps.sh "screentests:300:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'small_screen'" || exit 1
for round in 1 2; do
  for cfg in "base::" "scr::--option small_screen=1" "a3:kmerlsh_amd/lib_diag/libklsh_a3.so:--option small_screen=1" "a1:kmerlsh_amd/lib_diag/libklsh_a1.so:--option small_screen=1" "w3:kmerlsh_amd/lib_diag/libklsh_w3.so:--option small_screen=1"; do
    name=${cfg%%:*}; rest=${cfg#*:}; lib=${rest%%:*}; opt=${rest#*:}
    if [ -n "$lib" ]; then export KLSH_LIB=$lib; else unset KLSH_LIB; fi
    timeout -k 10 200 python bench.py --steps 4 --warmup 1 --cpu-baseline none $opt > gpurun_out/ab/${name}_$round.log 2>&1 || { echo "$name failed"; tail -3 gpurun_out/ab/${name}_$round.log; exit 1; }
    python3 -c "import json,sys; [print('$name $round', round(json.loads(l)['ms_per_step'],1), json.loads(l)['parity'].get('ok')) for l in open('gpurun_out/ab/${name}_$round.log') if l.startswith('{')]"
  done
done
