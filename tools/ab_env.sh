#!/usr/bin/env bash
# A/B of runtime environment settings on the parity headline in one GPU session:
#   ENVS="X=1 Y=2" (each word one arm; "-" = no extra setting) bash tools/ab_env.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:-"--no-cpu --no-densify --no-seeds --no-fast --steps 3 --warmup 1"}
i=0
for e in ${ENVS:--}; do
  i=$((i+1))
  if [ "$e" = "-" ]; then
    timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/abe_$i.log 2>&1; rc=$?
  else
    env $e timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/abe_$i.log 2>&1; rc=$?
  fi
  [ $rc -eq 0 ] || { echo "$e bench rc=$rc"; exit $rc; }
  tail -1 gpurun_out/abe_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e', d['value'], 'Mpatch/s', d['kernel_ms_per_launch'], 'ms E', d['E_mean_evals_per_patch'])"
done
