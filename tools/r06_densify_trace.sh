#!/usr/bin/env bash
# rocprofv3 kernel traces of the config-4 densify at one rank (tools/densify_trace.py),
# both protocols of dist.densify_partitioned_device, in the given refine modes
# (MODES="fast parity"); output gpurun_out/dtr06/<mode>_<protocol>/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for m in ${MODES:-fast}; do
  for p in ${PROTOCOLS:-device slots}; do
    D=gpurun_out/dtr06/${m}_$p
    mkdir -p $D
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $D -o run -- \
      python3 tools/densify_trace.py --mode $m --reps 3 --protocol $p > $D/log.txt 2>&1
    rc=$?; echo "$m $p rc=$rc"; grep '^{' $D/log.txt | tail -1; [ $rc -eq 0 ] || exit $rc
  done
done
