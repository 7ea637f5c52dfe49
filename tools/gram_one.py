#!/usr/bin/env python3
"""One int8-Gram variant, `--reps` launches, for rocprofv3 counter passes
(tools build; MMB_GRAM_I8_SHAPE / MMB_GRAM_I8_V1 / MMB_GRAM_DIAG from the
environment).  x: random t(5) rows (1M x 300 by default).

    MMB_GRAM_I8_SHAPE=5 python tools/gram_one.py --n 1000000 --reps 5
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
import mmb_lib  # noqa: E402

mmb_lib.load(os.path.join(ROOT, "tools", "diag", "libmmb_diag.so"))
import torch  # noqa: E402

import pipeline as P  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--reps", type=int, default=5)
args = ap.parse_args()
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(3)
x = (torch.randn(args.n, 300, generator=g, device=dev) * 0.3).contiguous()
cm = P.colmax(x)
ws = P.GramWorkspace(args.n, 300, dev)
G = torch.empty((300, 300), dtype=torch.float64, device=dev)
for _ in range(args.reps):
    P.gram_i8(x, cm, G, ws=ws)
torch.cuda.synchronize()
print("done", float(G[0, 0]))
