#!/usr/bin/env python3
"""Projection-kernel ablation in ONE process (CDNA guide §5.4 rule 24): the
bench-path projection (+ fused PC removal) under each MMB_PROJ_DIAG value,
interleaved over rounds; prints median / min ms per variant.

    python tools/proj_diag.py [--n N] [--rounds R] [--reps K] diag ...

diag bits (timing-only builds, wrong outputs): 1 no epilogue, 2 A chunk 0
only (L2-resident A), 4 B chunk 0 only, 8 no MFMAs; 0 = the real kernel.
A case "vK" or "vK:D" selects MMB_PROJ_VARIANT=K (with diag D); plain "D"
is the default variant.  Every diag-0 case must reproduce the default
kernel's rows bit for bit.
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
    ap.add_argument("diag", nargs="*", default=["0", "1", "2", "3", "8", "9"])
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    inp = synth.device_workload(args.n, 40, 400_000, seed=1, device=dev)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
    step = P.FusedStep(inp, gen.networks(), chunks=1, stream_project=False)
    step.run()
    torch.cuda.synchronize()
    pc = step.pc
    ref = step.mmb2.clone()
    del inp["audio"], inp["visual"]
    torch.cuda.empty_cache()
    cases = []
    for d in args.diag:
        if d.startswith("v"):
            v, _, dg = d[1:].partition(":")
            cases.append((v, dg or "0"))
        else:
            cases.append(("", d))
    res = {c: [] for c in cases}

    def run():
        P.mm2_project(step.s, step.x, step.aux, step.proj, out=step.mmb2, pc=pc, sif_out=step.sif)

    for _ in range(args.rounds):
        for variant, v in cases:
            os.environ.pop("MMB_PROJ_VARIANT", None)
            if variant:
                os.environ["MMB_PROJ_VARIANT"] = variant
            os.environ["MMB_PROJ_DIAG"] = v
            step.mmb2.zero_()
            run()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.reps):
                run()
            b.record()
            torch.cuda.synchronize()
            res[(variant, v)].append(a.elapsed_time(b) / args.reps)
            if v == "0":
                err = ((step.mmb2 - ref).abs().max()).item()
                assert err == 0.0, f"variant {variant or 'default'} output differs: {err}"
    os.environ.pop("MMB_PROJ_DIAG", None)
    os.environ.pop("MMB_PROJ_VARIANT", None)
    for (variant, v), t in res.items():
        print(f"variant={variant or 'default'} diag={v}: median {statistics.median(t):.4f} ms  "
              f"min {min(t):.4f} ms  {[round(x, 4) for x in t]}")


if __name__ == "__main__":
    main()
