#!/usr/bin/env python3
"""Same-process A/B of the MMB2 stream kernel at narrow frame widths (the
two-kernel step of FusedStep: stream -> s in HBM -> projection): the
narrow-frame kernel variants against utt_wave_kernel, selected per launch with
MMB_STREAM_NARROW in the tools build (libmmb_diag.so).  Interleaved rounds,
per-phase HIP event times, median per variant; outputs compared first.

    python tools/narrow_ab.py --T 20 --A 76 --Vd 48 --V 3016 --variants 0,2,3
"""
import argparse
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--T", type=int, default=20)
    ap.add_argument("--A", type=int, default=76)
    ap.add_argument("--Vd", type=int, default=48)
    ap.add_argument("--V", type=int, default=3016)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--variants", default="0,2,3")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    inp = synth.device_workload(args.n, args.T, args.V, A=args.A, Vd=args.Vd, seed=4000, device=dev)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, args.A, args.Vd, norm=None).to(dev)
    step = P.FusedStep(inp, gen.networks(), stream_project=False)
    variants = args.variants.split(",")
    outs = {}
    for v in variants:
        os.environ["MMB_STREAM_NARROW"] = v
        sif, mm2 = step.run()
        torch.cuda.synchronize()
        if int(v) < 6:  # 6-9: timing-only ablations (wrong rows, NaN x)
            step.check()
        step.reset()
        outs[v] = (step.x.clone(), mm2.clone(), sif.clone())
    base = outs[variants[0]]
    for v in variants[1:]:
        o = outs[v]
        print(f"variant {v} vs {variants[0]}: x equal {torch.equal(o[0], base[0])}, "
              f"mmb2 max abs diff {(o[1] - base[1]).abs().max().item():.3e}, "
              f"sif max abs diff {(o[2] - base[2]).abs().max().item():.3e}", flush=True)
    res = {v: {} for v in variants}
    for r in range(args.rounds):
        for v in variants:
            os.environ["MMB_STREAM_NARROW"] = v
            tr = {}
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                step.run(trace=tr)
            e1.record()
            torch.cuda.synchronize()
            res[v].setdefault("step", []).append(e0.elapsed_time(e1) / args.steps)
            for ph, evs in tr.items():
                res[v].setdefault(ph, []).append(sum(x.elapsed_time(y) for x, y in evs) / args.steps)
        print(f"round {r}: " + "  ".join(f"{v}: {res[v]['step'][-1]:.3f} ms" for v in variants), flush=True)
    for v in variants:
        print(f"variant {v}: " + ", ".join(f"{ph} {statistics.median(x):.3f}" for ph, x in res[v].items()))


if __name__ == "__main__":
    main()
