#!/usr/bin/env bash
# rocprofv3 profile of the performance-mode kernel (bench.py --mode fast): one
# kernel-trace/stats run, then separate --pmc passes (SQ issue/stall counters,
# LDS, FETCH/WRITE sizes).  Output under gpurun_out/fprof_<tag>/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-r02}
ARGS=${PROF_ARGS:-"--mode fast --cell 7 --steps 2 --warmup 1 --no-cpu --no-densify --no-seeds --no-fast"}
D=gpurun_out/fprof_$TAG
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $ARGS > $D/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $D/p$i -o run -- python3 bench.py $ARGS > $D/p$i.log 2>&1
  rc=$?; echo "pass $i ($line) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<LIST
${PASSES:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU_FP64 GRBM_GUI_ACTIVE
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH
FETCH_SIZE
WRITE_SIZE}
LIST
python3 tools/summarize_profile.py $D $D/summary.json > /dev/null && echo summarized
