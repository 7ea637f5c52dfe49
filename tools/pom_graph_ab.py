#!/usr/bin/env python3
"""configs[2]'s dataset splits (POM's real valid / test splits, g11) as HIP
graphs, per FusedStep variant: the split stream (mmb_mm2_stream_split) on or
off, the projection forked beside the PC solve or fused with the removal.
Host wall per replay incl. the sync (bench.py dataset_splits' measure),
median of --reps, alternated.  One JSON line.

    python tools/pom_graph_ab.py [--reps 40] [--dataset pom|mosi]
"""
import argparse
import json
import os
import statistics
import sys
import time

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

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--reps", type=int, default=40)
ap.add_argument("--dataset", default="pom")
ap.add_argument("--variants", default="split_fork,split_nofork,nosplit_fork,nosplit_nofork")
args = ap.parse_args()
dev = L.require_gpu()
if args.dataset == "pom":
    z = np.load(os.path.join(ROOT, "tests", "golden", "g11_pom_splits.npz"), allow_pickle=False)
    splits = synth.pom_splits(z["valid_ids"], z["test_ids"], z["weights"], int(z["table_seed"]))
    A, Vd = 300, 300
else:
    splits, A, Vd = synth.mosi_splits(), 76, 48
inps = [synth.to_device(sp, dev) for sp in splits]
torch.manual_seed(0)
gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(dev)
variants = {"split_fork": dict(), "split_nofork": dict(fork_projection=False),
            "nosplit_fork": dict(split_stream=False),
            "nosplit_nofork": dict(split_stream=False, fork_projection=False)}
graphs = {}
variants = {k: v for k, v in variants.items() if k in args.variants.split(",")}
for name, kw in variants.items():
    steps = [P.FusedStep(inp, gen.networks(), **kw) for inp in inps]
    graphs[name] = {"each": [P.StepGraph(st) for st in steps],
                    "concurrent": P.StepGraph(steps, concurrent=True),
                    "serial": P.StepGraph(steps, concurrent=False)}


def wall(g):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.run(check=True)
    return (time.perf_counter() - t0) * 1e3


res = {}
for r in range(args.reps):
    for name, gs in graphs.items():
        for si, g in enumerate(gs["each"]):
            res.setdefault(f"{name}_split{si}", []).append(wall(g))
        res.setdefault(f"{name}_concurrent", []).append(wall(gs["concurrent"]))
        res.setdefault(f"{name}_serial", []).append(wall(gs["serial"]))
print(json.dumps({k: round(statistics.median(v), 4) for k, v in res.items()}), flush=True)
