#!/usr/bin/env python3
"""VERDICT r03 item 5, measured before any kernel work: the performance mode's
CG refine with forward differences (the spec, oracle/or_fast.c) against the
same CG with the analytic gradient of the continuous objective
(tools/grad_experiment.c), on the CPU restatement.  Children of the
performance pipeline's own parents (raw seed patches -> fast refine at
n = 16), quality against the synthetic ground truth as bench.py reports it,
and the cost in evaluation-equivalents: an FD iteration is 5 evaluations
(3 forward differences + 2 probes); an analytic iteration is 2 probes plus one
evaluation-with-gradient, priced at `--grad-cost` evaluations (DESIGN.md
costs it at ~2.3 in the kernel's sampling passes).

    python tools/grad_experiment.py [--config cfg2_8view_1080p] [--parents 3000] [--cell 11]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import densepoints_amd as dp  # noqa: E402
from densepoints_amd import synth  # noqa: E402
from oracle import pyoracle as orc  # noqa: E402


def build(out):
    src = [os.path.join(ROOT, "oracle", f) for f in ("oracle.c", "or_seeds.c")]
    src.append(os.path.join(ROOT, "tools", "grad_experiment.c"))
    cmd = ["gcc", "-O2", "-std=c11", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-fopenmp", "-shared",
           "-I", os.path.join(ROOT, "oracle"), "-o", out, *src, "-lm"]
    subprocess.run(cmd, check=True)
    return out


def quality(cfg, kids, acc):
    k = kids[acc == 1]
    z, nrm = synth.surface(cfg, k["pos"][:, :2].astype(np.float64))
    nn = k["normal"].astype(np.float64)
    nn /= np.maximum(np.linalg.norm(nn, axis=1, keepdims=True), 1e-30)
    ang = np.degrees(np.arccos(np.clip(np.abs((nn * nrm).sum(1)), 0.0, 1.0)))
    dz = np.abs(k["pos"][:, 2] - z)
    return {"accepted": int(len(k)), "median_abs_dz": float(np.median(dz)), "p90_abs_dz": float(np.percentile(dz, 90)),
            "median_normal_err_deg": round(float(np.median(ang)), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2_8view_1080p")
    ap.add_argument("--parents", type=int, default=3000)
    ap.add_argument("--cell", type=int, default=11)
    ap.add_argument("--iters", default="2,3,4,5,6")
    ap.add_argument("--grad-cost", type=float, default=2.3)
    ap.add_argument("--qscale", type=float, default=0.0, help="> 0: per-sample derivatives rounded to 1/qscale")
    ap.add_argument("--noclamp", action="store_true", help="tap slopes also across clamped tile edges")
    a = ap.parse_args()
    lib = ctypes.CDLL(build("/tmp/libgradexp.so"))
    P_ = ctypes.c_void_p
    lib.exp_fast_expand_batch_an.argtypes = [P_, P_, ctypes.c_int, P_, P_, P_, P_]
    lib.exp_set.argtypes = [ctypes.c_double, ctypes.c_int]
    lib.exp_set(a.qscale, int(a.noclamp))
    cfg = synth.named(a.config)
    P, imgs, seeds = synth.scene_host(cfg)
    S = orc.Scene(P, imgs, dp.Options(expand_cell_size=a.cell))
    rng = np.random.default_rng(3)
    pick = np.sort(rng.choice(len(seeds), size=min(len(seeds), 3 * a.parents), replace=False))
    raw = S.seeds_to_patches(seeds[pick])
    ok = S.fast_refine(raw, 16)
    parents = np.ascontiguousarray(raw[ok == 1][: a.parents])
    out = {"config": a.config, "cell": a.cell, "parents": int(len(parents)), "grad_cost": a.grad_cost,
           "qscale": a.qscale, "noclamp": a.noclamp,
           "parents_quality": quality(cfg, parents, np.ones(len(parents), np.uint8))}
    for it in [int(x) for x in a.iters.split(",")]:
        fo = orc.fast_options(iters=it)
        kids, acc = S.fast_expand(parents, fo)
        E = kids["evals"].astype(np.float64)
        live = E > 0
        fd = {"E_mean": round(float(E[live].mean()), 3), **quality(cfg, kids, acc)}
        # FD cost: every evaluation costs 1 (the filter's included)
        fd["cost_eval_equiv"] = fd["E_mean"]
        kids2 = np.zeros_like(kids)
        acc2 = np.zeros_like(acc)
        st = (ctypes.c_long * 2)()
        lib.exp_fast_expand_batch_an(ctypes.c_void_p(S._h), parents.ctypes.data, len(parents), ctypes.byref(fo),
                                     kids2.ctypes.data, acc2.ctypes.data, st)
        nlive = int(live.sum())
        g_per, p_per = st[0] / max(nlive, 1), st[1] / max(nlive, 1)
        an = {"grad_evals_mean": round(g_per, 3), "probe_evals_mean": round(p_per, 3), **quality(cfg, kids2, acc2)}
        an["cost_eval_equiv"] = round(p_per + a.grad_cost * g_per + 1.0, 3)  # + the filter evaluation
        out[f"iters{it}"] = {"forward_differences": fd, "analytic": an}
        print(json.dumps({f"iters{it}": out[f"iters{it}"]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
