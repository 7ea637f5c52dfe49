#!/usr/bin/env python3
"""In-process A/B of the bench step: two kernels (stream -> HBM s ->
projection with the fused PC removal) vs the fused stream + projection
kernel (s in LDS; separate PC removal).  Interleaved rounds, per-phase HIP
event times, median per variant.

    python tools/fused_ab.py [--n 1000000] [--rounds 4] [--steps 3]
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
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--diags", default="",
                    help="comma list of MMB_FUSED_DIAG[:MMB_FUSED_UNR[:MMB_FUSED_PIPE]] values: "
                         "kernel-only timing of the fused kernel's ablations / streamer "
                         "load-group sizes / pipelined streamer beside the plain stream kernel")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    inp = synth.device_workload(args.n, 40, 400_000, seed=1, device=dev)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
    steps = {"two_kernel": P.FusedStep(inp, gen.networks(), stream_project=False),
             "fused": P.FusedStep(inp, gen.networks(), stream_project=True),
             "fused_pipe": P.FusedStep(inp, gen.networks(), stream_project=True)}
    pipe_of = {"two_kernel": "0", "fused": "0", "fused_pipe": "1"}
    for k, st in steps.items():
        os.environ["MMB_FUSED_PIPE"] = pipe_of[k]
        st.run()
    torch.cuda.synchronize()
    c = steps["fused_pipe"]
    print("pipelined streamer bit-identical:", torch.equal(steps["fused"].x, c.x),
          torch.equal(steps["fused"].mmb2, c.mmb2), torch.equal(steps["fused"].sif, c.sif), flush=True)
    for st in steps.values():
        st.check()
    a, b = steps["two_kernel"], steps["fused"]
    print("x equal:", torch.equal(a.x, b.x), " mmb2 max abs diff:",
          (a.mmb2 - b.mmb2).abs().max().item(), " sif max abs diff:",
          (a.sif - b.sif).abs().max().item(), flush=True)
    res = {k: {} for k in steps}
    for r in range(args.rounds):
        for k, st in steps.items():
            tr = {}
            os.environ["MMB_FUSED_PIPE"] = pipe_of[k]
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
    steps["fused"].check()
    if not args.diags:
        return
    inputs = dict(audio=inp["audio"], visual=inp["visual"], ids32=inp["ids"], table=inp["table"],
                  wtab32=inp["wtab"])

    def stream():
        P.mm2_stream(a.n, 40, 300, 300, 300, out=(a.x, a.s, a.aux), colmax=a.colmax,
                     colmax_ws=a.colmax_ws, **inputs)

    def fused():
        P.mm2_stream_project(b.n, 40, 300, 300, 300, proj=b.proj, out=(b.x, b.aux, b.mmb2),
                             colmax=b.colmax, colmax_ws=b.colmax_ws, **inputs)

    variants = [("stream", "0", stream), ("fused", "0", fused)]
    variants += [(f"fused diag:unr {d}", d, fused) for d in args.diags.split(",") if d]
    kt = {name: [] for name, _, _ in variants}
    for r in range(args.rounds):
        for name, dg, fn in variants:
            dg, _, rest = dg.partition(":")
            un, _, pp = rest.partition(":")
            os.environ["MMB_FUSED_DIAG"] = dg
            os.environ["MMB_FUSED_UNR"] = un or "8"
            os.environ["MMB_FUSED_PIPE"] = pp or "0"
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            kt[name].append(e0.elapsed_time(e1) / args.steps)
    os.environ["MMB_FUSED_DIAG"] = "0"
    os.environ["MMB_FUSED_UNR"] = "8"
    os.environ.pop("MMB_FUSED_PIPE", None)
    for name in kt:
        print(f"kernel {name}: median {statistics.median(kt[name]):.3f} ms  min {min(kt[name]):.3f}")


if __name__ == "__main__":
    main()
