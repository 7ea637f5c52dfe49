#!/usr/bin/env python3
"""Same-process A/B of the multi-workgroup PC solve (tools build, r05):
the r05 round (Cholesky beside the exchange of the raw product, 8 waves)
against the r04 round (MMB_PC_SOLVE_V1=1: Cholesky, then the exchange,
16 waves), HIP events around `reps` back-to-back solves of a bench-shaped
Gram (d = 300, k = 11, 7 power iterations), alternated over rounds; and the
two PCs against each other.

    python tools/pc_ab.py [--reps 200] [--rounds 5] [--iters 7] [--ablations]

(several --iters: the per-round cost is the slope over n_iter; --ablations
adds the r05 kernel without the round's update / factor / both, timing only)
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

import pipeline as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, nargs="+", default=[7])
    ap.add_argument("--ablations", action="store_true")
    ap.add_argument("--step-g", type=int, default=0,
                    help="solve the Gram (and Omega) of a bench-shaped FusedStep of this many rows "
                         "instead of the synthetic 4096 x 300 one")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(1)
    n, d, k = 4096, 300, 11
    if args.step_g:
        import models
        import synth
        inp = synth.device_shard(0, args.step_g, 40, 400_000, seed=1000, device=dev)
        torch.manual_seed(0)
        gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
        st = P.FusedStep(inp, gen.networks())
        st.run(check=True)
        G = st.G.clone()
        z0 = P.omega(d, k, dev).clone()
        ev = torch.linalg.eigvalsh(G.cpu())
        print(json.dumps({"step_rows": args.step_g, "eig_top12": [float(v) for v in ev.flip(0)[:12]]}), flush=True)
        del st, inp
    else:
        x = 0.4 * torch.randn(n, d, generator=g, dtype=torch.float64) + 0.3 * torch.randn(d, generator=g, dtype=torch.float64)
        G = (x.T @ x).to(dev)
        z0 = torch.randn(d, k, generator=g, dtype=torch.float64).to(dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    pc = torch.empty((1, d), dtype=torch.float64, device=dev)
    out = {}
    pcs = {}

    variants = {"new": {}, "v1": {"MMB_PC_SOLVE_V1": "1"}}
    if args.ablations:  # timing only: the round without its update (1), factor (2), both (3)
        variants.update({f"abl{a}": {"MMB_PC_ABL": str(a)} for a in (1, 2, 3)})

    def run(name, it):
        for key in ("MMB_PC_SOLVE_V1", "MMB_PC_ABL"):
            os.environ.pop(key, None)
        os.environ.update(variants[name])
        P.pc_solve(G, z0, 1, False, n_iter=it, out=pc, flag=flag)
        torch.cuda.synchronize()
        pcs[(name, it)] = pc.clone()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.reps):
            P.pc_solve(G, z0, 1, False, n_iter=it, out=pc, flag=flag)
        b.record()
        torch.cuda.synchronize()
        out.setdefault(f"{name}_iter{it}", []).append(round(a.elapsed_time(b) * 1e3 / args.reps, 2))

    for _ in range(args.rounds):
        for it in args.iters:
            for name in variants:
                run(name, it)
    for key in ("MMB_PC_SOLVE_V1", "MMB_PC_ABL"):
        os.environ.pop(key, None)
    res = {"us_per_solve": out, "us_min": {k_: min(v) for k_, v in out.items()},
           "flag": int(flag.item()),
           "pc_maxdiff_new_vs_v1": {str(it): float((pcs[("new", it)] - pcs[("v1", it)]).abs().max())
                                    for it in args.iters}}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
