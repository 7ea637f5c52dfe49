#!/usr/bin/env python3
"""Where the narrow fused kernel's cold text rows come from (r05): the MOSI
bench step (1M utterances, T 20, A 76, Vd 48, V 3016) with its ids as drawn
(Zipf(1.1): ~42 % of the tokens miss the 32 LDS-resident hot words and read
their 2.4 KB text-cache rows from L2 / Infinity Cache), then with every cold
id folded into ranks 33..400 (the cold rows then span 0.9 MB: L2-resident)
and into rank 33 alone (one row) -- the hot / cold split and everything else
unchanged.  Kernel and step times (HIP events), alternated over rounds.

    python tools/nf_cold_ab.py [--n 1000000] [--steps 5] [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
import torch  # noqa: E402

import models  # noqa: E402
import pipeline as P  # noqa: E402
import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    inp = synth.device_workload(args.n, 20, 3016, A=76, Vd=48, seed=4000, device=dev)
    ids0 = inp["ids"]
    hot = 32
    variants = {"zipf": ids0,
                "cold_in_400": torch.where(ids0 > hot, hot + 1 + (ids0 - hot - 1) % 368, ids0),
                "cold_one_row": torch.where(ids0 > hot, torch.full_like(ids0, hot + 1), ids0)}
    cold_frac = float((ids0 > hot).float().mean())
    steps = {}
    for name, ids in variants.items():
        torch.manual_seed(0)
        gen = models.AudioVisualGeneratorMultimodal(300, 76, 48, norm=None).to(dev)
        steps[name] = P.FusedStep({**inp, "ids": ids}, gen.networks(), narrow_fused=True)
    res = {k: {"kernel": [], "step": []} for k in variants}
    for _ in range(args.rounds):
        for name, st in steps.items():
            for _ in range(3):
                st.run()
            torch.cuda.synchronize()
            for _ in range(args.steps):
                tr = {}
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                st.run(trace=tr)
                b.record()
                torch.cuda.synchronize()
                res[name]["kernel"].append(sum(x.elapsed_time(y) for x, y in tr["mm2_stream_project_narrow"]))
                res[name]["step"].append(a.elapsed_time(b))
            st.check()
    print(json.dumps({"n": args.n, "cold_token_fraction": round(cold_frac, 4),
                      **{k: {m: round(statistics.median(v), 4) for m, v in d.items()} for k, d in res.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
