#!/usr/bin/env bash
# A/B of the partitioned densify's generation protocols (scaling_leg, config 4,
# one rank): r05 (one host wait per generation) vs r04, alternated twice.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for i in 1 2; do
  for p in r05 r04; do
    timeout -k 10 400 python -u bench.py --steps 2 --no-fast --no-seeds --no-cpu --densify-steps 3 \
      --densify-protocol $p > gpurun_out/abproto_${p}_$i.log 2>&1
    rc=$?; echo "$p $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python - "$p" gpurun_out/abproto_${p}_$i.log <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
s = j["scaling_leg"]
for m in ("parity", "fast"):
    r = s[m]
    print(sys.argv[1], m, r["Mpatches_per_s"], r["ms_per_densify"], "refine", r["refine_ms_max_rank"],
          "non_refine", r["non_refine_ms"], r["phase_ms_max_rank"], r["store_crc32"])
print("densify_e2e", j["densify_e2e"]["wall_s"], j["densify_e2e"]["refine_ms"], j["densify_e2e_fast"]["wall_s"],
      j["densify_e2e_fast"]["refine_ms"])
PY
  done
done
