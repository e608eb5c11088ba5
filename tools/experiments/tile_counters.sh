#!/usr/bin/env bash
# Parity-kernel LDS tiles: rate and wave-cycle / TA counters
# of bench.py's parity headline for the default library and the variants built
# from r05_parity_lds_tiles.patch (libdp_pad4k.so: 3 waves/SIMD, HBM taps;
# libdp_tiles.so: 3 waves/SIMD, LDS tiles), plus the tile path statistics
# (libdp_tstats.so).  Output: gpurun_out/tiles/.
set -u
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
D=gpurun_out/tiles
mkdir -p $D
ARGS="--no-fast --no-densify --no-seeds --no-cpu --steps 3 --warmup 1"
for v in ${VARIANTS:-libdensepoints.so libdp_pad4k.so libdp_tiles.so}; do
  DP_LIB_VARIANT=$v timeout -k 10 300 python -u bench.py $ARGS > $D/bench_$v.log 2>&1
  rc=$?; echo "$v bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
  DP_LIB_VARIANT=$v timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE TA_TA_BUSY_sum --kernel-trace --output-format csv \
    -d $D/pmc_$v -o run -- python3 bench.py $ARGS > $D/pmc_$v.log 2>&1
  rc=$?; echo "$v pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
DP_LIB_VARIANT=libdp_tstats.so timeout -k 10 300 python -u tools/experiments/tile_stats.py > $D/tstats.log 2>&1
rc=$?; echo "tstats rc=$rc"; exit $rc
