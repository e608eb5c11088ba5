#!/usr/bin/env python3
"""Static audit of one kernel instance's gfx950 disassembly (the counts quoted
in DESIGN.md §5a "the instructions the compiler added"): compiles a source with
the library's flags to device assembly and prints, per loop (LLVM's
"Loop: Header=... Depth=..." block annotations), the VALU instruction count,
the SGPR-spill reloads (v_readlane_b32 from the VGPRs the kernel's
v_writelane_b32 spills use), quarter-rate integer multiplies and
boolean round trips (v_cndmask 0/1 feeding a compare).

    python tools/isa_audit.py [--src densepoints_amd/csrc/dp_kernels.hip]
                              [--kernel 'refine_kernelILi4ELi2E']

Static counts: a block inside a loop counts once however often it runs.
"""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load_build():
    import importlib.util
    spec = importlib.util.spec_from_file_location("_dp_build", os.path.join(ROOT, "densepoints_amd", "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def disassemble(src):
    B = load_build()
    flags = [f for f in B.FLAGS if f not in ("-shared", "-fPIC")]
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run([B.hipcc(), *flags, "--cuda-device-only", "-S", "-o", out, src], check=True,
                       cwd=os.path.dirname(src), stderr=subprocess.DEVNULL)
        return open(out).read().split("\n")


def instance(lines, pattern):
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l)]
    for k, i in enumerate(starts):
        if re.search(pattern, lines[i]):
            end = starts[k + 1] if k + 1 < len(starts) else len(lines)
            return lines[i].split(":")[0], lines[i:end]
    raise SystemExit("no kernel matches %r" % pattern)


def audit(body):
    spill_vgprs = {m.group(1) for l in body for m in [re.match(r"\s*v_writelane_b32 (v\d+), s\d+, \d+", l)] if m}
    loop = ("", 0)
    per = collections.defaultdict(collections.Counter)
    prev = ""
    for l in body:
        m = re.match(r"^(\.LBB\d+_\d+):\s*(;.*)?$", l)
        if m:
            c = m.group(2) or ""
            d = re.search(r"Depth=(\d+)", c)
            h = re.search(r"Header=(\w+)", c)
            loop = (h.group(1) if h else "", int(d.group(1)) if d else 0)
            continue
        s = l.strip()
        if not s.startswith("v_"):
            continue
        c = per[loop]
        c["valu"] += 1
        m = re.match(r"v_readlane_b32 s\d+, (v\d+), \d+", s)
        if m and m.group(1) in spill_vgprs:
            c["spill_reloads"] += 1
        if s.startswith("v_writelane_b32"):
            c["spill_writes"] += 1
        if s.startswith(("v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_mad_i64_i32")):
            c["wide_int_mul"] += 1
        if re.match(r"v_cmp_ne_u32_e\d+ \S+, 0, (v\d+)", s) and re.match(r"v_cndmask_b32_e64 v\d+, 0, 1,", prev):
            c["bool_round_trips"] += 1
        prev = s
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default=os.path.join(ROOT, "densepoints_amd", "csrc", "dp_kernels.hip"))
    ap.add_argument("--kernel", default=r"refine_kernelILi4ELi2E")
    args = ap.parse_args()
    name, body = instance(disassemble(os.path.abspath(args.src)), args.kernel)
    per = audit(body)
    tot = collections.Counter()
    print(name)
    print("%-14s %5s %6s %14s %13s %13s %17s" % ("loop header", "depth", "VALU", "spill reloads", "spill writes",
                                                "wide int mul", "bool round trips"))
    for (h, d), c in sorted(per.items(), key=lambda x: (x[0][1], x[0][0])):
        tot.update(c)
        print("%-14s %5d %6d %14d %13d %13d %17d" % (h or "-", d, c["valu"], c["spill_reloads"], c["spill_writes"],
                                                     c["wide_int_mul"], c["bool_round_trips"]))
    print("%-14s %5s %6d %14d %13d %13d %17d" % ("total", "", tot["valu"], tot["spill_reloads"], tot["spill_writes"],
                                                 tot["wide_int_mul"], tot["bool_round_trips"]))


if __name__ == "__main__":
    main()
