#!/usr/bin/env python3
"""Generate tests/golden/seeds_small.npz: fixed inputs and the oracle's output
of every stage of seed generation (Features::Matcher::GenerateSeeds,
modules/features/matcher.cpp:18-474) on a small synthetic scene.

OpenCV (ORB, BFMatcher) and Eigen are absent from the image, so these are
restatement vectors, not reference outputs (DESIGN.md "Seed generation"):
they freeze oracle/or_seeds.c between rounds (the CPU suite re-runs it) and
are the GPU suite's target for the HIP path.

Inputs are stored, not regenerated: 3 views of 320x240 BGR8 (rendered by the
product's synthetic renderer at generation time only) and their projection
matrices.  Options: 3000 features, 4 levels, FAST threshold 8 (the synthetic
texture is low-contrast), everything else the reference defaults.

A second fixture, seeds_akaze_small.npz, holds the same stages with
DetectorType::AKAZE (oracle/or_akaze.c; threshold 0.0002 for the
low-contrast texture, 64-byte descriptor rows) on seeds_small.npz's inputs.

usage: python tests/golden/make_golden_seeds.py   (rewrites both fixtures)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from densepoints_amd import synth  # noqa: E402
from oracle import pyoracle  # noqa: E402

OPTIONS = {"n_features": 3000, "n_levels": 4, "fast_threshold": 8}
AKAZE_OPTIONS = {"detector_type": 0, "akaze_threshold": 0.0002}


def generate(options=OPTIONS, inputs=None):
    if inputs is None:
        cfg = synth.config(3, 320, 240, 1)
        P, imgs, _ = synth.scene_host(cfg)
    else:
        P, imgs = inputs
    r = pyoracle.seeds_run(P, imgs, pyoracle.matcher_options(**options))
    out = {"P": P.astype(np.float64), "images": np.stack(imgs).astype(np.uint8)}
    c = r["counts"]
    out["counts"] = np.array([c[k] for k in ("detected", "keypoints", "ratio_matches", "matches", "points")],
                             dtype=np.int64)
    out["kp_count"] = np.array([len(k) for k in r["keypoints"]], dtype=np.int64)
    out["keypoints"] = np.concatenate(r["keypoints"])
    out["descriptors"] = np.concatenate(r["descriptors"])
    out["pairs"] = np.array(r["pairs"], dtype=np.int32)
    out["q2t"] = np.concatenate(r["q2t"])
    out["points"] = r["points"]
    return out


if __name__ == "__main__":
    import sys

    if "--akaze-only" in sys.argv:
        # regenerate the AKAZE fixture alone, on the committed seeds_small.npz inputs
        g = np.load(os.path.join(HERE, "seeds_small.npz"))
        out = {"P": g["P"], "images": g["images"]}
    else:
        out = generate()
        np.savez_compressed(os.path.join(HERE, "seeds_small.npz"), **out)
        print({k: v.shape for k, v in out.items()}, out["counts"])
    ak = generate(AKAZE_OPTIONS, (out["P"], list(out["images"])))
    del ak["P"], ak["images"]  # the inputs are seeds_small.npz's
    np.savez_compressed(os.path.join(HERE, "seeds_akaze_small.npz"), **ak)
    print({k: v.shape for k, v in ak.items()}, ak["counts"])
