#!/usr/bin/env python3
"""Dataset-split step variants (tools build, r05): eager FusedStep runs of the
real POM splits (g11: 100 x 1089 and 203 x 1357 tokens) and MOSI's three,
per MMB_STREAM_SMALL variant of the workgroup stream kernel for a few long
rows (0: the large-N kernel, 1: 320 threads x 16 frame / 8 text rows in
flight, 2: 1024 threads x 4 / 4), alternated; median phase times (HIP events).

    python tools/splits_ab.py [--reps 20]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
import mmb_lib  # noqa: E402

mmb_lib.load(os.path.join(ROOT, "tools", "diag", "libmmb_diag.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import models  # noqa: E402
import pipeline as P  # noqa: E402
import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=20)
args = ap.parse_args()
dev = torch.device("cuda", 0)
z = np.load(os.path.join(ROOT, "tests", "golden", "g11_pom_splits.npz"), allow_pickle=False)
splits = synth.pom_splits(z["valid_ids"], z["test_ids"], z["weights"], int(z["table_seed"]))
torch.manual_seed(0)
gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
steps = [P.FusedStep(synth.to_device(sp, dev), gen.networks()) for sp in splits]
res = {}
ref = {}
for r in range(3):
    for v in ("0", "1", "2"):
        os.environ["MMB_STREAM_SMALL"] = v
        for si, st in enumerate(steps):
            for _ in range(args.reps):
                tr = {}
                st.run(trace=tr)
                torch.cuda.synchronize()
                ms = sum(a.elapsed_time(b) for a, b in tr["mm2_stream"])
                res.setdefault(f"split{si}_v{v}", []).append(ms)
            st.check()
            if r == 0:
                ref.setdefault(si, {})[v] = st.sif.clone()
out = {k: round(statistics.median(x), 4) for k, x in res.items()}
for si in ref:
    for v in ("1", "2"):
        d = (ref[si][v] - ref[si]["0"]).abs().max().item() / ref[si]["0"].abs().max().item()
        out[f"split{si}_v{v}_sif_maxrel_vs_v0"] = d
print(json.dumps(out), flush=True)
