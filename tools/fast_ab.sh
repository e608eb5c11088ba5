#!/usr/bin/env bash
# GPU: the performance-mode suite, then the bench's perf_mode sub-object
# (parity headline + n = 7 / 11), summarised in one line per window.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fast.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_fast.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_fast.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu --no-densify --no-seeds ${BENCH_EXTRA:-} > gpurun_out/b1.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/b1.log; exit $rc; }
python3 tools/bench_summary.py gpurun_out/b1.log
