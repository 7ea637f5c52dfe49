#!/usr/bin/env python3
"""Kernel-only timing of the fused stream + projection kernel's ablations at
any workload shape (tools build: MMB_FUSED_DIAG / _UNR / _PIPE knobs).

    python tools/fused_shape_ab.py --T 20 --A 76 --Vd 48 --V 3016 \
        --variants 0::2,1::2,8::0,0::0

A variant is DIAG[:UNR[:PIPE]]: 0::2 the product kernel, 1::2 its streamers
alone (the projectors only hand the ring slots back), 8::0 the projectors
alone (constant sums, group-at-a-time streamer), 0::0 the group-at-a-time
streamer.  Interleaved rounds, median per variant.
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
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
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--T", type=int, default=20)
    ap.add_argument("--A", type=int, default=76)
    ap.add_argument("--Vd", type=int, default=48)
    ap.add_argument("--V", type=int, default=3016)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--variants", default="0::2,1::2,8::0,0::0")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    inp = synth.device_workload(args.n, args.T, args.V, A=args.A, Vd=args.Vd, seed=4000, device=dev)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, args.A, args.Vd, norm=None).to(dev)
    st = P.FusedStep(inp, gen.networks(), stream_project=True)
    st.run()
    torch.cuda.synchronize()
    st.check()
    kw = dict(audio=inp["audio"], visual=inp["visual"], ids32=inp["ids"], table=inp["table"],
              wtab32=inp["wtab"])

    def fused():
        P.mm2_stream_project(st.n, args.T, 300, args.A, args.Vd, proj=st.proj, out=(st.x, st.aux, st.mmb2),
                             colmax=st.colmax, colmax_ws=st.colmax_ws, **kw)

    names = [v for v in args.variants.split(",") if v]
    kt = {v: [] for v in names}
    for r in range(args.rounds):
        for v in names:
            dg, _, rest = v.partition(":")
            un, _, pp = rest.partition(":")
            os.environ["MMB_FUSED_DIAG"] = dg or "0"
            os.environ["MMB_FUSED_UNR"] = un or "8"
            os.environ["MMB_FUSED_PIPE"] = pp or "2"
            fused()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                fused()
            e1.record()
            torch.cuda.synchronize()
            kt[v].append(e0.elapsed_time(e1) / args.steps)
        print(f"round {r}: " + "  ".join(f"{v} {kt[v][-1]:.3f}" for v in names), flush=True)
    for v in names:
        print(f"variant {v}: median {statistics.median(kt[v]):.3f} ms  min {min(kt[v]):.3f}")


if __name__ == "__main__":
    main()
