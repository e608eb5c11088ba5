#!/usr/bin/env bash
# Round-6 GPU check: selected test files (TESTS="tests/a.py tests/b.py", or
# ALL=1 for the whole GPU suite), smoke(), then optionally a bench line
# (BENCH_ARGS).  Every GPU step has its own time limit; any failure stops.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${TAG:-r06}
if [ "${ALL:-0}" = 1 ]; then
  TESTS=tests
fi
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/${tag}_pytest.log)"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${SMOKE:-1}" = 1 ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/${tag}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/${tag}_smoke.log)"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py $BENCH_ARGS > gpurun_out/${tag}_bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/${tag}_bench.log; echo; [ $rc -eq 0 ] || exit $rc
fi
exit 0
