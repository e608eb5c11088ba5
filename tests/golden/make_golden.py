#!/usr/bin/env python3
"""Generate tests/golden/pmvs_small.npz: fixed inputs and the oracle's outputs
for every stage of the patch loop on a small synthetic scene.

The reference itself cannot be built here (OpenCV contrib, PCL,
Eigen and GTest are absent), so these vectors are produced by the CPU
restatement in oracle/. That restatement is pinned by the reference's own
known answers (tests/test_oracle_kat.py). The fixture freezes its
behaviour: the CPU suite re-runs the oracle against it (regressions), and
the GPU suite runs the HIP path against it.

Inputs are stored, not regenerated: 4 views of 192x144 BGR8 (the images come
from the product's synthetic renderer at generation time only), the 4
projection matrices and the seed points.

usage: python tests/golden/make_golden.py   (rewrites pmvs_small.npz)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from densepoints_amd import synth  # noqa: E402
from oracle import pyoracle  # noqa: E402

MODES = {"eval": 0, "filter": 1, "nm": 2, "seed": 3, "expand": 4}


def generate():
    cfg = synth.config(4, 192, 144, 1)
    cfg.seed_stride_px = 12.0
    P, imgs, seeds = synth.scene_host(cfg)
    S = pyoracle.Scene(P, imgs)
    out = {"P": P.astype(np.float64), "images": np.stack(imgs).astype(np.uint8), "seeds": seeds.astype(np.float64)}
    pat = S.seeds_to_patches(seeds)
    out["seed_patches"] = pat
    for cell in (16, 11, 7):
        for name in ("filter", "nm", "seed"):
            r = pat.copy()
            acc = S.refine(r, cell, MODES[name], 1)
            out[f"refine_{name}_{cell}"] = r
            out[f"accept_{name}_{cell}"] = acc.astype(np.uint8)
    seeded = pat.copy()
    acc = S.refine(seeded, 16, MODES["seed"], 1)
    parents = seeded[acc != 0]
    out["expand_parents"] = parents
    kids, kacc = S.expand(parents, 1)
    out["expand_children"] = kids
    out["expand_accept"] = kacc.astype(np.uint8)
    dense, st = S.densify(seeds)
    out["densify"] = dense
    out["densify_stats"] = np.array([st["patches"], st["seed_patches"], st["pops"]], dtype=np.int64)
    return out


def main():
    out = generate()
    path = os.path.join(HERE, "pmvs_small.npz")
    np.savez_compressed(path, **out)
    print(path, os.path.getsize(path), "bytes;",
          {k: (v.shape, str(v.dtype)[:20]) for k, v in out.items() if k not in ("images",)})


if __name__ == "__main__":
    main()
