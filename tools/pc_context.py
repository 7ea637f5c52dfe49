#!/usr/bin/env python3
"""Why the PC solve runs slower inside a step than back to back (r06: 69.8 us
in the 125k step's kernel trace, 56.5 us alone): the solve timed by HIP
events right after different kinds of preceding work on the same stream --
nothing (back to back), a 1 GiB copy (HBM-bound, caches flushed), a 64 MiB
write (the L2s flushed, the MALL not), a large bf16 GEMM (MFMA-bound), an
idle device sleep (clock ramp) -- median over --reps.  One JSON line.

    python tools/pc_context.py [--reps 50]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
import torch  # noqa: E402

import mmb_lib as L  # noqa: E402
import pipeline as P  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=50)
args = ap.parse_args()
dev = L.require_gpu()
g = torch.Generator(device="cpu").manual_seed(1)
x = 0.4 * torch.randn(4096, 300, generator=g, dtype=torch.float64) + 0.3 * torch.randn(300, generator=g, dtype=torch.float64)
G = (x.T @ x).to(dev)
z0 = P.omega(300, 11, dev).clone()
flag = torch.zeros(1, dtype=torch.int32, device=dev)
pc = torch.empty((1, 300), dtype=torch.float64, device=dev)
ws = P.solve_workspace(300, dev)
big_a = torch.empty(1 << 28, dtype=torch.float32, device=dev)  # 1 GiB
big_b = torch.empty_like(big_a)
mid = torch.empty(1 << 24, dtype=torch.float32, device=dev)  # 64 MiB
ma = torch.randn(8192, 8192, dtype=torch.bfloat16, device=dev)
mb = torch.randn(8192, 8192, dtype=torch.bfloat16, device=dev)
mc = torch.empty(8192, 8192, dtype=torch.bfloat16, device=dev)


def solve():
    P.pc_solve(G, z0, 1, False, out=pc, flag=flag, ws=ws)


pre = {"back_to_back": None,
       "after_copy_1GiB": lambda: big_b.copy_(big_a),
       "after_write_64MiB": lambda: mid.fill_(1.0),
       "after_bf16_gemm": lambda: torch.mm(ma, mb, out=mc),
       "after_sleep": lambda: torch.cuda._sleep(2_000_000)}
out = {}
for name, fn in pre.items():
    for _ in range(5):
        if fn:
            fn()
        solve()
    torch.cuda.synchronize()
    ts = []
    for _ in range(args.reps):
        if fn:
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        solve()
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    us = [a.elapsed_time(b) * 1e3 for a, b in ts]
    out[name] = {"median_us": round(statistics.median(us), 2), "min_us": round(min(us), 2)}
out["flag"] = int(flag.item())
print(json.dumps(out), flush=True)
