#!/usr/bin/env python3
"""The f64 Gram of a dataset split (mmb_gram -> gram_small_kernel for n <=
4096) timed alone: HIP events around --reps back-to-back launches, for the
MOSI split sizes (1284 / 686 / 229 rows) and POM's (100 / 203), d = 300.

    python tools/gram_small_time.py [--reps 200]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
import torch  # noqa: E402

import mmb_lib as L  # noqa: E402
import pipeline as P  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=200)
args = ap.parse_args()
dev = L.require_gpu()
out = {}
for n in (1284, 686, 229, 203, 100):
    x = torch.randn(n, 300, device=dev)
    G = torch.empty(300, 300, dtype=torch.float64, device=dev)
    ws = P.GramWorkspace(n, 300, dev)
    P.gram(x, None, G, ws=ws)
    torch.cuda.synchronize()
    ref = (x.double().T @ x.double())
    err = float((G - ref).abs().max() / ref.abs().max())
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.reps):
            P.gram(x, None, G, ws=ws)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / args.reps)
    out[str(n)] = {"us": round(min(ts), 2), "rel_err_vs_torch_f64": err}
print(json.dumps(out), flush=True)
