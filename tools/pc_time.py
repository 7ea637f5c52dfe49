#!/usr/bin/env python3
"""The product library's PC solve (mmb_pc_solve_mc: pc_solve_mc_kernel with
its squaring workgroups since r06b) timed alone and checked against the oracle:
HIP events around --reps back-to-back solves at n_iter = 7, for a synthetic
4096 x 300 Gram (tools/pc_ab.py's), a bench-step Gram (--step-g rows) and
the transposed branch of POM's real valid split (100 rows).  One JSON line:
us per solve and max |pc - oracle pc_from_gram|.

    python tools/pc_time.py [--reps 200] [--step-g 125000]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mmb_lib as L  # noqa: E402

# --lib PATH: an A/B clone of the product library (tools/ab_libs), loaded
# explicitly before the mirror modules bind to it
_lib = next((sys.argv[i + 1] for i, a in enumerate(sys.argv[:-1]) if a == "--lib"), None)
if _lib:
    L.load(_lib)
import models  # noqa: E402
import pipeline as P  # noqa: E402
import synth  # noqa: E402
from oracle import sif_oracle as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--reps", type=int, default=200)
ap.add_argument("--step-g", type=int, default=125_000)
args = ap.parse_args()
dev = L.require_gpu()
cases = {}
g = torch.Generator(device="cpu").manual_seed(1)
x = 0.4 * torch.randn(4096, 300, generator=g, dtype=torch.float64) + 0.3 * torch.randn(300, generator=g, dtype=torch.float64)
cases["synthetic4096"] = ((x.T @ x).to(dev), P.omega(300, 11, dev).clone(), False)
torch.manual_seed(0)
gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
inp = synth.device_shard(0, args.step_g, 40, 400_000, seed=1000, device=dev)
st = P.FusedStep(inp, gen.networks())
st.run(check=True)
cases[f"step{args.step_g}"] = (st.G.clone(), P.omega(300, 11, dev).clone(), False)
del st, inp
z = np.load(os.path.join(ROOT, "tests", "golden", "g11_pom_splits.npz"), allow_pickle=False)
sp = synth.to_device(synth.pom_splits(z["valid_ids"], z["test_ids"], z["weights"], int(z["table_seed"]))[0], dev)
st = P.FusedStep(sp, gen.networks())
st.run(check=True)
n = sp["ids"].shape[0]
om = P.omega(n, 11, dev).contiguous()
cases["pom_valid_transposed"] = (st.G.clone(), P.xt_omega(st.x, None, om), True)
out = {}
flag = torch.zeros(1, dtype=torch.int32, device=dev)
pc = torch.empty((1, 300), dtype=torch.float64, device=dev)
for name, (G, z0, tr) in cases.items():
    P.pc_solve(G, z0, 1, tr, out=pc, flag=flag)
    torch.cuda.synchronize()
    ref = O.pc_from_gram(G.cpu().numpy(), z0.cpu().numpy(), 1, tr)
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.reps):
            P.pc_solve(G, z0, 1, tr, out=pc, flag=flag)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / args.reps)
    out[name] = {"us": round(min(ts), 2), "maxdiff_vs_oracle": float(np.abs(pc.cpu().numpy() - ref).max())}
out["flag"] = int(flag.item())
print(json.dumps(out), flush=True)
