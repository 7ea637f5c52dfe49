#!/usr/bin/env python3
"""The PC solve (mmb_pc_solve_mc) warm and cold (r05): HIP events around
each of `reps` solves of a bench-shaped Gram (d = 300, k = 11, 7 power
iterations), run back to back (code and data L2-resident) or each after a
512 MB copy that sweeps L2 and the Infinity Cache (the solve's place in the
step: after the fused kernel's stream).  One library per process:

    python tools/pc_cold_ab.py [--lib multimodal-baselines_amd/libmmb.so] [--reps 50]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
import mmb_lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(ROOT, "multimodal-baselines_amd", "libmmb.so"))
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    mmb_lib.load(os.path.abspath(args.lib))
    import torch
    import pipeline as P

    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(1)
    n, d, k = 4096, 300, 11
    x = 0.4 * torch.randn(n, d, generator=g, dtype=torch.float64) + 0.3 * torch.randn(d, generator=g, dtype=torch.float64)
    G = (x.T @ x).to(dev)
    z0 = torch.randn(d, k, generator=g, dtype=torch.float64).to(dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    pc = torch.empty((1, d), dtype=torch.float64, device=dev)
    src = torch.empty(128 << 20, dtype=torch.float32, device=dev).uniform_()
    dst = torch.empty_like(src)
    res = {}
    for mode in ("warm", "cold", "warm", "cold"):
        ts = []
        P.pc_solve(G, z0, 1, False, n_iter=7, out=pc, flag=flag)
        for _ in range(args.reps):
            if mode == "cold":
                dst.copy_(src)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            P.pc_solve(G, z0, 1, False, n_iter=7, out=pc, flag=flag)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        res.setdefault(mode, []).append(round(statistics.median(ts), 2))
    print(json.dumps({"lib": os.path.basename(args.lib), "us_median": res, "flag": int(flag.item()),
                      "pc0": float(pc[0, 0])}), flush=True)


if __name__ == "__main__":
    main()
