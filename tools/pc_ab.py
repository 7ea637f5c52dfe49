#!/usr/bin/env python3
"""Same-process A/B of the multi-workgroup PC solve (tools build, r05):
the r05 round (Cholesky beside the exchange of the raw product, 8 waves)
against the r04 round (MMB_PC_SOLVE_V1=1: Cholesky, then the exchange,
16 waves), HIP events around `reps` back-to-back solves of a bench-shaped
Gram (d = 300, k = 11, 7 power iterations), alternated over rounds; and the
two PCs against each other.

    python tools/pc_ab.py [--reps 200] [--rounds 5]
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
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(1)
    n, d, k = 4096, 300, 11
    x = 0.4 * torch.randn(n, d, generator=g, dtype=torch.float64) + 0.3 * torch.randn(d, generator=g, dtype=torch.float64)
    G = (x.T @ x).to(dev)
    z0 = torch.randn(d, k, generator=g, dtype=torch.float64).to(dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    pc = torch.empty((1, d), dtype=torch.float64, device=dev)
    out = {"new": [], "v1": []}
    pcs = {}

    def run(name):
        if name == "v1":
            os.environ["MMB_PC_SOLVE_V1"] = "1"
        else:
            os.environ.pop("MMB_PC_SOLVE_V1", None)
        P.pc_solve(G, z0, 1, False, out=pc, flag=flag)
        torch.cuda.synchronize()
        pcs[name] = pc.clone()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.reps):
            P.pc_solve(G, z0, 1, False, out=pc, flag=flag)
        b.record()
        torch.cuda.synchronize()
        out[name].append(round(a.elapsed_time(b) * 1e3 / args.reps, 2))

    for _ in range(args.rounds):
        for name in ("new", "v1"):
            run(name)
    os.environ.pop("MMB_PC_SOLVE_V1", None)
    res = {"us_per_solve": out, "us_min": {k_: min(v) for k_, v in out.items()},
           "flag": int(flag.item()),
           "pc_maxdiff_new_vs_v1": float((pcs["new"] - pcs["v1"]).abs().max())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
