#!/usr/bin/env python3
"""Same-process A/B of whole steps at any workload shape: the fused stream +
projection step against the two-kernel step (stream kernel -> s in HBM ->
projection with the fused PC removal).  Interleaved rounds, per-phase HIP
event times, median per variant.

    python tools/step_ab.py --T 20 --A 76 --Vd 48 --V 3016 [--n 1000000]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-baselines_amd"))

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
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    inp = synth.device_workload(args.n, args.T, args.V, A=args.A, Vd=args.Vd, seed=4000, device=dev)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, args.A, args.Vd, norm=None).to(dev)
    steps = {"fused": P.FusedStep(inp, gen.networks(), stream_project=True),
             "two_kernel": P.FusedStep(inp, gen.networks(), stream_project=False)}
    for st in steps.values():
        st.run()
    torch.cuda.synchronize()
    for st in steps.values():
        st.check()
    a, b = steps["fused"], steps["two_kernel"]
    print("x equal:", torch.equal(a.x, b.x), " mmb2 max abs diff:", (a.mmb2 - b.mmb2).abs().max().item(),
          flush=True)
    res = {k: {} for k in steps}
    for r in range(args.rounds):
        for k, st in steps.items():
            tr = {}
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                st.run(trace=tr)
            e1.record()
            torch.cuda.synchronize()
            res[k].setdefault("step", []).append(e0.elapsed_time(e1) / args.steps)
            for ph, evs in tr.items():
                res[k].setdefault(ph, []).append(sum(x.elapsed_time(y) for x, y in evs) / args.steps)
        print(f"round {r}: " + "  ".join(f"{k} {res[k]['step'][-1]:.3f} ms" for k in steps), flush=True)
    for k in steps:
        print(k + ": " + ", ".join(f"{ph} {statistics.median(v):.3f}" for ph, v in res[k].items()))


if __name__ == "__main__":
    main()
