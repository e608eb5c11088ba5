"""In-tree build of libdensepoints.so (gfx950) -- no JIT cache, no pip install.

hipcc compiles the kernels and the host-side C ABI in one shared object.
-ffp-contract=off is part of the parity spec: every fp64/f32 expression of the
arithmetic spec is one IEEE rounding on both the CPU and CDNA4.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "lib", "libdensepoints.so")
SOURCES = ["dp_capi.hip", "dp_kernels.hip", "dp_filter.hip", "dp_seeds.hip", "dp_seeds_capi.hip", "dp_orb.hip",
           "dp_fast.hip", "dp_akaze.hip", "dp_bfs.hip"]
HEADERS = ["dp_internal.h", "dp_geom.h", "dp_detmath.h", "dp_synth.h", "dp_devmath.h", "dp_ctx.h", "dp_dlt.h",
           "dp_seeds.h", "dp_orb.h", "dp_orb_pattern.h", "dp_akaze.h"]
ARCH = os.environ.get("DP_OFFLOAD_ARCH", "gfx950")
FLAGS = [
    "-O3",
    "-std=c++17",
    f"--offload-arch={ARCH}",
    "-ffp-contract=off",
    "-fno-fast-math",
    "-fPIC",
    "-shared",
    "-Wall",
    "-Wno-unused-value",
    "-Wno-unused-result",
    # MFMA results in VGPRs (gfx950's unified register file): the knnMatch
    # epilogue reads every accumulator with VALU, so the AGPR form would add one
    # v_accvgpr_read per element (the refine kernels have no MFMA)
    "-mllvm",
    "-amdgpu-mfma-vgpr-form=1",
]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def _stamp_text() -> str:
    return " ".join(FLAGS)


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    # the default library records the flags it was built with: a variant build
    # copied over it (or a flag change here) makes it stale even when newer
    try:
        with open(OUT + ".flags") as f:
            if f.read() != _stamp_text():
                return True
    except OSError:
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps += [os.path.join(HERE, "..", "include", h) for h in ("densepoints.h", "densepoints_probe.h")]
    deps.append(__file__)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False) -> str:
    """One object per source, compiled in parallel (hipcc -c), then linked
    into the shared object; an object is rebuilt when its source, a header or
    this file is newer."""
    extra = os.environ.get("DP_EXTRA_FLAGS", "").split()
    if not force and not extra and not _stale():
        return OUT
    # variant builds (DP_EXTRA_FLAGS) keep their objects apart
    tag = "obj" if not extra else "obj_" + hashlib.sha1(" ".join(extra).encode()).hexdigest()[:10]
    objdir = os.path.join(HERE, "lib", tag)
    os.makedirs(objdir, exist_ok=True)
    cflags = [f for f in FLAGS if f != "-shared"]
    common = [os.path.join(CSRC, h) for h in HEADERS] + [__file__]
    common += [os.path.join(HERE, "..", "include", h) for h in ("densepoints.h", "densepoints_probe.h")]
    t_common = max(os.path.getmtime(d) for d in common if os.path.exists(d))
    procs, objs = [], []
    for s in SOURCES:
        src, obj = os.path.join(CSRC, s), os.path.join(objdir, s.replace(".hip", ".o"))
        objs.append(obj)
        if not force and os.path.exists(obj) and \
                os.path.getmtime(obj) > max(os.path.getmtime(src), t_common):
            continue
        cmd = [hipcc(), *cflags, *extra, "-c", "-o", obj + ".tmp", src]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((subprocess.Popen(cmd, cwd=CSRC), obj))
    failed = False
    for pr, obj in procs:
        if pr.wait() != 0:
            failed = True
        else:
            os.replace(obj + ".tmp", obj)
    if failed:
        raise RuntimeError("hipcc failed")
    # DP_LIB_NAME: a variant's file name under lib/ (loaded by DP_LIB_VARIANT);
    # a variant (DP_EXTRA_FLAGS) never takes the default name: without
    # DP_LIB_NAME it is named after its flags' hash
    name = os.environ.get("DP_LIB_NAME") or ("libdensepoints_%s.so" % tag[4:] if extra else os.path.basename(OUT))
    out = os.path.join(os.path.dirname(OUT), name)
    if extra and os.path.abspath(out) == os.path.abspath(OUT):
        raise RuntimeError("DP_EXTRA_FLAGS builds must not overwrite %s (set DP_LIB_NAME)" % OUT)
    tmp = out + ".tmp"
    subprocess.run([hipcc(), *FLAGS, *extra, "-o", tmp, *objs], check=True, cwd=CSRC)
    os.replace(tmp, out)
    # only the default library's own build records the default flags (a
    # DP_LIB_NAME link elsewhere leaves the default library -- and its stamp -- alone)
    if not extra and os.path.abspath(out) == os.path.abspath(OUT):
        with open(OUT + ".flags", "w") as f:
            f.write(_stamp_text())
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
