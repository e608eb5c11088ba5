#!/usr/bin/env bash
# rocprofv3 evidence for bench.py's roofline objects, one workload per call:
#   tools/r05_profile.sh parity|fast7|fast11
# a --kernel-trace --stats run, then separate --pmc passes (SQ issue counters
# with GRBM_GUI_ACTIVE; wave-cycle split; VALU mix; FETCH_SIZE; WRITE_SIZE: MI355X_MICROARCH.md's per-pass
# limits) of the same bench command; lines starting with "?" are optional passes.  Output: gpurun_out/prof_r06/<workload>/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
W=${1:?workload}
BASE="--steps 3 --warmup 1 --no-cpu --no-densify --no-seeds --no-fast"
case $W in
  parity) ARGS="$BASE" ;;
  fast7) ARGS="--mode fast --cell 7 $BASE" ;;
  fast11) ARGS="--mode fast --cell 11 $BASE" ;;
  *) echo "unknown workload $W"; exit 2 ;;
esac
D=gpurun_out/prof_r06/$W
mkdir -p $D
ARGS="$ARGS --detail $D/detail.json"
echo "$ARGS" > $D/args.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py $ARGS > $D/trace.log 2>&1
rc=$?; echo "$W trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  opt=0
  case $line in "?"*) opt=1; line=${line#?} ;; esac
  timeout -s KILL 240 rocprofv3 --pmc $line --kernel-trace --output-format csv -d $D/pmc$i -o run -- python3 bench.py $ARGS > $D/pmc$i.log 2>&1
  rc=$?; echo "$W pass $i ($line) rc=$rc"
  # a pass marked "?" (counters not known to exist on gfx950) may fail alone
  [ $rc -eq 0 ] || [ $opt -eq 1 ] || exit $rc
done <<LIST
SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64
FETCH_SIZE
WRITE_SIZE
?SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_LDS TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE
LIST
