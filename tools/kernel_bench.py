#!/usr/bin/env python3
"""Per-kernel microbenchmark on synthetic device data (for rocprofv3 passes).

    python tools/kernel_bench.py {stream,gram,project,project32,pcsolve,remove,all} [--n N] [--reps R]

Prints the mean HIP-event time per launch of each selected kernel.
"""
import argparse
import os
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


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", nargs="+")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--t", type=int, default=40)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--ids", default="zipf", choices=["zipf", "uniform", "hot", "seq"])
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    inp = synth.device_workload(args.n, args.t, 400_000, seed=1, device=dev)
    if args.ids == "uniform":
        inp["ids"].random_(1, 400_000)
    elif args.ids == "hot":
        inp["ids"].fill_(1)
    elif args.ids == "seq":  # each utterance reads a contiguous run of rows
        base = (torch.arange(args.n, device=dev, dtype=torch.int64) * args.t) % (400_000 - args.t)
        inp["ids"].copy_((base[:, None] + torch.arange(args.t, device=dev)[None, :] + 1).to(torch.int32))
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
    step = P.FusedStep(inp, gen.networks(), chunks=1, stream_project=False)
    step.run()
    torch.cuda.synchronize()
    which = set(args.which)
    if "all" in which:
        which = {"stream", "gram", "project", "project32", "pcsolve", "remove"}
    cnt = step.aux[0]
    z0 = P.omega(300, 11, dev)
    res = {}
    if "stream" in which:
        res["stream"] = timed(lambda: P.mm2_stream(step.n, step.t, 300, 300, 300, inp["audio"],
                                                   inp["visual"], ids32=inp["ids"],
                                                   table=inp["table"], wtab32=inp["wtab"],
                                                   out=(step.x, step.s, step.aux)), args.reps)
    if "stream_cm" in which:  # with the column bounds for the int8 Gram
        res["stream_cm"] = timed(lambda: P.mm2_stream(step.n, step.t, 300, 300, 300, inp["audio"],
                                                      inp["visual"], ids32=inp["ids"],
                                                      table=inp["table"], wtab32=inp["wtab"],
                                                      out=(step.x, step.s, step.aux),
                                                      colmax=step.colmax, colmax_ws=step.colmax_ws),
                                 args.reps)
    if "gram" in which:
        res["gram"] = timed(lambda: P.gram(step.x, None, step.G, ws=step.gws), args.reps)
    if "gram_i8" in which:  # int8-sliced Gram (+ the column bounds pass it needs)
        cm = P.colmax(step.x)
        Gi = torch.empty_like(step.G)
        res["colmax"] = timed(lambda: P.colmax(step.x, out=cm), args.reps)
        res["gram_i8"] = timed(lambda: P.gram_i8(step.x, cm, Gi, ws=step.gws), args.reps)
        G64 = P.gram(step.x, None, ws=step.gws)
        torch.cuda.synchronize()
        print(f"gram_i8 vs f64 Gram: max rel {((Gi - G64).abs().max() / G64.abs().max()).item():.3e}")
        Gref = Gi.clone()
        for dg in os.environ.get("GRAM_DIAGS", "").split(","):  # timing-only ablations
            if dg:
                os.environ["MMB_GRAM_DIAG"] = dg
                res[f"gram_i8 diag {dg}"] = timed(lambda: P.gram_i8(step.x, cm, Gi, ws=step.gws), args.reps)
                if int(dg) & 15 == 0:  # schedule variants: the same Gram
                    torch.cuda.synchronize()
                    print(f"gram_i8 diag {dg} bit-identical: {torch.equal(Gi, Gref)}")
        os.environ.pop("MMB_GRAM_DIAG", None)
    if "pcsolve" in which:
        res["pcsolve"] = timed(lambda: P.pc_solve(step.G, z0, 1, False), args.reps)
    if "remove" in which:
        pc = P.pc_solve(step.G, z0, 1, False)
        res["remove"] = timed(lambda: P.remove_pc(step.x, None, pc, out=step.sif), args.reps)
    if "project" in which:
        res["project"] = timed(lambda: P.mm2_project(step.s, step.x, step.aux, step.proj,
                                                     out=step.mmb2), args.reps)
    if "project_rm" in which:  # the bench path: projection + fused PC removal
        pc = P.pc_solve(step.G, z0, 1, False)
        res["project_rm"] = timed(lambda: P.mm2_project(step.s, step.x, step.aux, step.proj,
                                                        out=step.mmb2, pc=pc, sif_out=step.sif),
                                  args.reps)
    if "project32" in which:
        s32 = P.s_buffer(step.n, step.proj.kp, False, dev)
        P.mm2_stream(step.n, step.t, 300, 300, 300, inp["audio"], inp["visual"], ids32=inp["ids"],
                     table=inp["table"], wtab32=inp["wtab"], s_half=False,
                     out=(step.x, s32, step.aux))
        res["project32"] = timed(lambda: P.mm2_project(s32, step.x, step.aux, step.proj,
                                                       out=step.mmb2), args.reps)
    for k, v in res.items():
        print(f"{k}: {v:.4f} ms")




def pcsolve_breakdown():
    """pc_solve time vs n_iter (subspace iterations) on a 1M-row Gram."""
    dev = torch.device("cuda", 0)
    inp = synth.device_workload(200_000, 40, 100_000, A=4, Vd=4, seed=1, device=dev)
    num, cnt = P.weighted_sum(inp["table"], inp["ids"], wtab32=inp["wtab"])
    G = P.gram(num, cnt)
    z0 = P.omega(300, 11, dev)
    for it in (0, 1, 7):
        print(f"pc_solve n_iter={it}: {timed(lambda: P.pc_solve(G, z0, 1, False, n_iter=it), 5):.4f} ms")


if __name__ == "__main__":
    if sys.argv[1:2] == ["pcsolve_breakdown"]:
        pcsolve_breakdown()
    else:
        main()
