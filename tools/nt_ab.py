#!/usr/bin/env python3
"""Cross-step cache A/B (tools build, r05): does the PC removal's traffic
evict the Zipf-hot word rows the NEXT step's fused kernel would find in L2 /
MALL?  The bench step at --n rows (125k: an 8-GPU rank's share of configs[3];
1M), `--steps` consecutive steps per variant (default removal vs
MMB_PC_REMOVE_NT=1: x read and rows written non-temporally), alternated over
rounds; per variant the median fused-kernel and step times (HIP events).

    python tools/nt_ab.py --n 125000 --steps 10 --rounds 4
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
import torch  # noqa: E402

import models  # noqa: E402
import pipeline as P  # noqa: E402
import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, nargs="+", default=[125_000, 1_000_000])
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--rounds", type=int, default=4)
args = ap.parse_args()
dev = torch.device("cuda", 0)
out = {}
for n in args.n:
    inp = synth.device_shard(0, n, 40, 400_000, seed=1000, device=dev)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
    st = P.FusedStep(inp, gen.networks())
    st.run(check=True)
    res = {"default": {"fused": [], "step": []}, "remove_nt": {"fused": [], "step": []}}
    for _ in range(args.rounds):
        for name in res:
            if name == "remove_nt":
                os.environ["MMB_PC_REMOVE_NT"] = "1"
            else:
                os.environ.pop("MMB_PC_REMOVE_NT", None)
            for k in range(args.steps):
                tr = {}
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                st.run(trace=tr)
                b.record()
                torch.cuda.synchronize()
                if k >= 2:  # the first steps after a switch carry the other variant's cache state
                    res[name]["fused"].append(sum(x.elapsed_time(y) for x, y in tr["mm2_stream_project"]))
                    res[name]["step"].append(a.elapsed_time(b))
    os.environ.pop("MMB_PC_REMOVE_NT", None)
    st.check()
    out[str(n)] = {k: {m: round(statistics.median(v), 4) for m, v in d.items()} for k, d in res.items()}
    print(json.dumps({"n": n, **out[str(n)]}), flush=True)
    del st, inp
    torch.cuda.empty_cache()
