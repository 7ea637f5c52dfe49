#!/usr/bin/env python3
"""Same-process A/B of the int8 Gram kernels (tools build, r05).

    python tools/gram_ab.py [--n 1000000 125000] [--reps 20] [--rounds 3]

x = the a2 rows of a bench-shaped FusedStep (1M x 300, Zipf ids), so the
column bounds are the step's own.  Per size: the round-4 kernel
(MMB_GRAM_I8_V1=1: per-k-step f64 updates), the level-sum kernel in each
shape (MMB_GRAM_I8_SHAPE 0 = product: three feature-group parts, slicing
staggered between SIMD partners; 1: four triangle runs; 2: three triangle
runs, spilling; 3: the product with LDS reads free to cross tiles; 4: with
the next tile's first B digit prefetched; 5: unstaggered) and
the product shape's
timing-only ablations (MMB_GRAM_DIAG 1 no MFMAs, 4 no slicing, 12 no slicing
and no x loads, 13 only barriers / LDS / epilogue), and 84 / 85 row ranges
(252 / 255 workgroups, the parts of a range then on different XCDs;
MMB_GRAM_RANGES) instead of 80, and x staged in LDS by DMA (MMB_GRAM_I8_SHAPE
6: gram_i8s_kernel, with its ablations), alternated over rounds;
HIP events around `reps` back-to-back calls (kernel + range reduction).
Also each variant's max |G - G_f64| / max |G_f64| against the exact f64 Gram.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
import mmb_lib  # noqa: E402

mmb_lib.load(os.path.join(ROOT, "tools", "diag", "libmmb_diag.so"))
import torch  # noqa: E402

import models  # noqa: E402
import pipeline as P  # noqa: E402
import synth  # noqa: E402

VARIANTS = {
    "v1_r04": {"MMB_GRAM_I8_V1": "1"},
    "levels_groups3_stagger": {},
    "levels_runs4x6": {"MMB_GRAM_I8_SHAPE": "1"},
    "levels_runs3x8": {"MMB_GRAM_I8_SHAPE": "2"},
    "levels_groups3_sb": {"MMB_GRAM_I8_SHAPE": "3"},
    "levels_groups3_pf": {"MMB_GRAM_I8_SHAPE": "4"},
    "levels_groups3_plain": {"MMB_GRAM_I8_SHAPE": "5"},
    "abl_no_mfma": {"MMB_GRAM_DIAG": "1"},
    "abl_no_slice": {"MMB_GRAM_DIAG": "4"},
    "abl_no_slice_no_load": {"MMB_GRAM_DIAG": "12"},
    "abl_skeleton": {"MMB_GRAM_DIAG": "13"},
    "ranges84": {"MMB_GRAM_RANGES": "84"},
    "ranges85": {"MMB_GRAM_RANGES": "85"},
    "staged": {"MMB_GRAM_I8_SHAPE": "6"},
    "staged_no_mfma": {"MMB_GRAM_I8_SHAPE": "6", "MMB_GRAM_DIAG": "1"},
    "staged_no_slice": {"MMB_GRAM_I8_SHAPE": "6", "MMB_GRAM_DIAG": "4"},
    "staged_no_slice_no_dma": {"MMB_GRAM_I8_SHAPE": "6", "MMB_GRAM_DIAG": "12"},
}


def with_env(kv, fn):
    old = {k: os.environ.get(k) for k in ("MMB_GRAM_I8_V1", "MMB_GRAM_I8_SHAPE", "MMB_GRAM_DIAG",
                                          "MMB_GRAM_RANGES")}
    for k in old:
        os.environ.pop(k, None)
    os.environ.update(kv)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[1_000_000, 125_000])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", nargs="+", default=None, help="a subset of VARIANTS (the product always)")
    args = ap.parse_args()
    variants = {k: v for k, v in VARIANTS.items()
                if args.variants is None or k in args.variants or k == "levels_groups3_stagger"}
    dev = torch.device("cuda", 0)
    nmax = max(args.n)
    inp = synth.device_workload(nmax, 40, 400_000, seed=1, device=dev)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
    step = P.FusedStep(inp, gen.networks())
    step.run(check=True)
    torch.cuda.synchronize()
    xall = step.x
    del inp
    out = {}
    for n in args.n:
        x = xall[:n].contiguous()
        cm = P.colmax(x)
        ws = P.GramWorkspace(n, 300, dev)
        G64 = P.gram(x, None, ws=ws).clone()
        G = torch.empty_like(G64)
        res = {}
        Gp = None
        for name, kv in variants.items():
            with_env(kv, lambda: P.gram_i8(x, cm, G, ws=ws))
            torch.cuda.synchronize()
            if name == "levels_groups3_stagger":
                Gp = G.clone()
            res[name] = {"err_vs_f64": float((G - G64).abs().max() / G64.abs().max()), "ms": [],
                         "same_as_product": None if Gp is None else bool(torch.equal(G, Gp))}
        for _ in range(args.rounds):
            for name, kv in variants.items():
                res[name]["ms"].append(round(with_env(kv, lambda: timed(
                    lambda: P.gram_i8(x, cm, G, ws=ws), args.reps)), 4))
        for name in res:
            res[name]["ms_min"] = min(res[name]["ms"])
        out[str(n)] = res
        print(json.dumps({"n": n, **{k: (v["ms_min"], v["err_vs_f64"], v["same_as_product"])
                                     for k, v in res.items()}}),
              flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
