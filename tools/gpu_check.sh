#!/usr/bin/env bash
# GPU session: build, parity tests, short bench. Each GPU step has its own time
# limit; a fault/abort/timeout (rc >= 124 or signal) stops the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
ok_rc() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo "build failed"; exit 3; }
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
ok_rc $rc || exit $rc
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc
