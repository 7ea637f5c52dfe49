#!/usr/bin/env python3
"""The bench step at --n rows (product library), `--steps` untraced steps
after a warm-up, for a kernel trace:

    rocprofv3 --kernel-trace --stats -d OUT -o step -- python3 tools/step_prof.py --n 125000

then `python3 tools/step_prof.py --gaps OUT/.../step_kernel_trace.csv` prints
each kernel's median duration and the median idle gap before it (r05: where
the per-rank step's time goes between the kernels).
"""
import argparse
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]


def gaps(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    rows.sort()
    per = {}
    for i, (s, e, n) in enumerate(rows):
        g = s - rows[i - 1][1] if i else 0
        per.setdefault(n, {"dur": [], "gap": []})
        per[n]["dur"].append(e - s)
        per[n]["gap"].append(g)
    out = {n: {"calls": len(v["dur"]), "dur_us": round(statistics.median(v["dur"]) / 1e3, 2),
               "gap_before_us": round(statistics.median(v["gap"]) / 1e3, 2)} for n, v in per.items()}
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=125_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--gaps", default=None)
    args = ap.parse_args()
    if args.gaps:
        gaps(args.gaps)
        return
    import mmb_lib
    mmb_lib.load()
    import torch

    import models
    import pipeline as P
    import synth
    dev = torch.device("cuda", 0)
    inp = synth.device_shard(0, args.n, 40, 400_000, seed=1000, device=dev)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
    st = P.FusedStep(inp, gen.networks())
    for _ in range(3):
        st.run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(args.steps):
        st.run()
    b.record()
    torch.cuda.synchronize()
    st.check()
    print(json.dumps({"n": args.n, "ms_per_step": round(a.elapsed_time(b) / args.steps, 4)}), flush=True)


if __name__ == "__main__":
    main()
