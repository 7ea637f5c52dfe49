#!/usr/bin/env python3
"""MOSI-shape two-kernel step: the projection (+ fused PC removal) phase under the
tools build's timing-only MMB_PROJ_DIAG ablations (wrong rows).  Same process,
interleaved rounds, median ms of the projection phase per setting."""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-baselines_amd"))
DIAG_LIB = os.environ.get("MMB_TOOLS_LIB", os.path.join(ROOT, "tools", "diag", "libmmb_diag.so"))
import mmb_lib  # noqa: E402

mmb_lib.load(DIAG_LIB)  # the tools build: explicit, never through the product loader
import torch  # noqa: E402

import models  # noqa: E402
import pipeline as P  # noqa: E402
import synth  # noqa: E402

dev = torch.device("cuda", 0)
inp = synth.device_workload(1_000_000, 20, 3016, A=76, Vd=48, seed=4000, device=dev)
torch.manual_seed(0)
gen = models.AudioVisualGeneratorMultimodal(300, 76, 48, norm=None).to(dev)
step = P.FusedStep(inp, gen.networks())
res = {}
settings = sys.argv[1:] or ["0", "1", "2", "4", "8"]
for r in range(3):
    for v in settings:
        os.environ["MMB_PROJ_DIAG"] = v
        tr = {}
        for _ in range(3):
            step.run(trace=tr)
        torch.cuda.synchronize()
        ph = [k for k in tr if k.startswith("mm2_project")][0]
        res.setdefault(v, []).append(sum(a.elapsed_time(b) for a, b in tr[ph]) / len(tr[ph]))
for v in settings:
    print(f"MMB_PROJ_DIAG={v}: projection phase median {statistics.median(res[v]):.3f} ms")
