set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_seeds.py tests/test_cli.py -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/r06_gputest2.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dev -o run -- python3 tools/densify_trace.py --mode fast --reps 3 --protocol device > gpurun_out/r06_trace_dev.log 2>&1 || exit 2
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_slots -o run -- python3 tools/densify_trace.py --mode fast --reps 3 --protocol slots > gpurun_out/r06_trace_slots.log 2>&1 || exit 3
