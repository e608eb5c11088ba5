#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (the check behind DESIGN's
"no spills" statements).  Usage: tools/resource_usage.py [source.hip ...]
[--filter fast_kernel]; compiles each source for gfx950 with the library's
flags into a temporary object and prints one line per kernel."""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from densepoints_amd import build as B  # noqa: E402


def usage(src, extra=()):
    flags = [f for f in B.FLAGS if f != "-shared"]
    with tempfile.TemporaryDirectory() as td:
        cmd = [B.hipcc(), *flags, *extra, "-c", "-o", os.path.join(td, "x.o"), src,
               "-Rpass-analysis=kernel-resource-usage"]
        out = subprocess.run(cmd, capture_output=True, text=True, cwd=os.path.dirname(src)).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(.*?): (\S+) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2)
        if k == "Function Name":
            cur = {"kernel": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sources", nargs="*", default=[os.path.join(B.CSRC, "dp_fast.hip")])
    ap.add_argument("--filter", default="")
    ap.add_argument("-D", action="append", default=[], help="extra -D defines")
    a = ap.parse_args()
    for src in a.sources:
        for r in usage(os.path.abspath(src), ["-D" + d for d in a.D]):
            if a.filter not in r["kernel"]:
                continue
            name = subprocess.run(["c++filt"], input=r["kernel"], capture_output=True, text=True).stdout.strip()
            name = re.sub(r"dpk::\(anonymous namespace\)::", "", name)
            print("%-70s VGPR %4s  SGPR %4s  scratch %4s  vspill %3s  sspill %3s  waves %s  LDS %s" % (
                name[:70], r.get("VGPRs", "?"), r.get("TotalSGPRs", "?"), r.get("ScratchSize [bytes/lane]", "?"),
                r.get("VGPRs Spill", "?"), r.get("SGPRs Spill", "?"), r.get("Occupancy [waves/SIMD]", "?"),
                r.get("LDS Size [bytes/block]", "?")))


if __name__ == "__main__":
    main()
