"""Debug helper: run one fast-mode configuration on the GPU and the oracle and
print the first differing patches field by field (tests/ conventions)."""
import sys

import torch  # HIP runtime first, as tests/conftest.py does

if torch.cuda.device_count() > 0:
    torch.cuda.init()
import numpy as np  # noqa: E402

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import densepoints_amd as dp  # noqa: E402
from densepoints_amd import _native as N  # noqa: E402
from test_gpu_parity import scene  # noqa: E402
from oracle import pyoracle as orc  # noqa: E402

cell = int(sys.argv[1]) if len(sys.argv) > 1 else 16
mode = N.MODE_FAST_REFINE
opts = {}
for kv in sys.argv[2:]:
    k, v = kv.split("=")
    opts[k] = float(v) if k in ("fd_step", "ls_step") else int(v)

sc = scene("hf6")
fo = dp.FastOptions(**opts)
with dp.Engine(device=0) as eng:
    eng.set_views(sc.views)
    eng.set_fast_options(fo)
    S = orc.Scene(sc.P, sc.imgs)
    seeds = sc.seeds[:200]
    gp = eng.seeds_to_patches(seeds)
    op = S.seeds_to_patches(seeds)
    ga = eng.fast_refine(gp, cell, mode)
    oa = S.fast_refine(op, cell, mode, orc.fast_options(fo))
bad = np.flatnonzero((ga != oa) | (gp.view(np.uint8).reshape(len(gp), -1) != op.view(np.uint8).reshape(len(op), -1)).any(1))
print("mismatching patches", bad[:20], len(bad))
for i in bad[:3]:
    for f in gp.dtype.names:
        if gp[f][i].tobytes() != op[f][i].tobytes():
            print(i, f, "gpu", gp[f][i], "oracle", op[f][i])
    print(i, "input", seeds[i] if i < len(seeds) else None)
    print(i, "accept", ga[i], oa[i], "evals", gp["evals"][i], op["evals"][i])
