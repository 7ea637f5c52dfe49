#!/usr/bin/env python3
"""In-process A/B of stream-kernel variants (MMB_STREAM_POLICY values, read
per launch): one workload, the variants interleaved over several rounds
(cdna_hip_programming.md §5.4 rule 24), median and min per variant.

    python tools/stream_ab.py 5 13 [--rounds 5] [--reps 5] [--ids zipf|uniform]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the MMB_* knobs these runs flip live in the tools build (make -C multimodal-baselines_amd/csrc diag)
DIAG_LIB = os.environ.get("MMB_TOOLS_LIB", os.path.join(ROOT, "tools", "diag", "libmmb_diag.so"))
sys.path.insert(0, os.path.join(ROOT, "multimodal-baselines_amd"))
import mmb_lib  # noqa: E402

mmb_lib.load(DIAG_LIB)  # the tools build: explicit, never through the product loader

import torch  # noqa: E402

import models  # noqa: E402
import pipeline as P  # noqa: E402
import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("policies", nargs="+")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ids", default="zipf", choices=["zipf", "uniform"])
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    inp = synth.device_workload(args.n, 40, 400_000, seed=1, device=dev)
    if args.ids == "uniform":
        inp["ids"].random_(1, 400_000)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
    step = P.FusedStep(inp, gen.networks(), chunks=1, stream_project=False)
    step.run()
    torch.cuda.synchronize()

    def launch():
        P.mm2_stream(step.n, step.t, 300, 300, 300, inp["audio"], inp["visual"], ids32=inp["ids"],
                     table=inp["table"], wtab32=inp["wtab"], out=(step.x, step.s, step.aux),
                     colmax=step.colmax, colmax_ws=step.colmax_ws)

    ref = None
    times = {p: [] for p in args.policies}
    for r in range(args.rounds):
        for p in args.policies:
            os.environ["MMB_STREAM_POLICY"] = p
            launch()
            torch.cuda.synchronize()
            if r == 0:  # every variant writes the same rows
                out = (step.x.clone(), step.s.clone(), step.aux.clone())
                if ref is None:
                    ref = out
                else:
                    same = all(torch.equal(a, b) for a, b in zip(ref, out))
                    print(f"policy {p}: outputs {'bit-identical' if same else 'DIFFER'}", flush=True)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.reps):
                launch()
            b.record()
            torch.cuda.synchronize()
            times[p].append(a.elapsed_time(b) / args.reps)
        print(f"round {r}: " + " ".join(f"{p}={times[p][-1]:.3f}" for p in args.policies), flush=True)
    for p in args.policies:
        print(f"policy {p}: median {statistics.median(times[p]):.3f} ms  min {min(times[p]):.3f} ms")


if __name__ == "__main__":
    main()
