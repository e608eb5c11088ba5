#!/usr/bin/env bash
# rocprofv3 kernel-trace summary of the bench (no counters), then separate PMC
# passes for HBM traffic.  Output under gpurun_out/prof_<tag>/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS=${PROF_ARGS:-"--steps 3 --warmup 1 --no-cpu --no-densify --no-seeds"}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG/trace -o run -- python3 bench.py $ARGS > gpurun_out/prof_$TAG/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
if [ -n "${PMC:-1}" ]; then
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_$TAG/pmc_fetch -o run -- python3 bench.py $ARGS > gpurun_out/prof_$TAG/pmc_fetch.log 2>&1
  rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_$TAG/pmc_write -o run -- python3 bench.py $ARGS > gpurun_out/prof_$TAG/pmc_write.log 2>&1
  rc=$?; echo "pmc write rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
find gpurun_out/prof_$TAG -name "*.csv" | head -20
