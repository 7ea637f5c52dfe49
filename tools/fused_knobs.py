#!/usr/bin/env python3
"""Kernel-only timing of mmb_mm2_stream_project under environment knob
settings (the library reads MMB_FUSED_* per launch), interleaved rounds in
one process, median per setting.  Outputs are checked bit-identical to the
first setting unless a setting contains DIAG.

    python tools/fused_knobs.py "MMB_FUSED_PIPE=1" "MMB_FUSED_PIPE=1,MMB_FUSED_PSLEEP=8" ...
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
    ap.add_argument("settings", nargs="+")
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--t", type=int, default=40)
    ap.add_argument("--ragged", action="store_true", help="Poisson(40) lengths in [1, 64] (T = 64)")
    ap.add_argument("--uniform", action="store_true", help="token ids uniform over [1, V)")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    t = 64 if args.ragged else args.t
    inp = synth.device_workload(args.n, t, 400_000, seed=1, device=dev,
                                poisson_len=40.0 if args.ragged else None)
    if args.uniform:
        inp["ids"].random_(1, 400_000)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
    st = P.FusedStep(inp, gen.networks(), stream_project=True)
    st.run()
    torch.cuda.synchronize()
    kw = dict(audio=inp["audio"], visual=inp["visual"], ids32=inp["ids"], table=inp["table"],
              wtab32=inp["wtab"])
    outs = [torch.empty_like(st.x), torch.empty_like(st.aux), torch.empty_like(st.mmb2)]

    def fused():
        P.mm2_stream_project(st.n, t, 300, 300, 300, proj=st.proj, out=outs, colmax=st.colmax,
                             colmax_ws=st.colmax_ws, **kw)

    base = os.environ.copy()

    def apply(setting):
        os.environ.clear()
        os.environ.update(base)
        for kv in filter(None, setting.split(",")):
            k, _, v = kv.partition("=")
            os.environ[k] = v

    ref = None
    kt = {s: [] for s in args.settings}
    for r in range(args.rounds):
        for s in args.settings:
            apply(s)
            fused()
            torch.cuda.synchronize()
            if r == 0 and "DIAG" not in s:
                cur = [o.clone() for o in outs]
                if ref is None:
                    ref = cur
                else:
                    same = all(torch.equal(torch.nan_to_num(a), torch.nan_to_num(b))
                               for a, b in zip(ref, cur))
                    print(f"{s}: bit-identical to {args.settings[0]}: {same}", flush=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                fused()
            e1.record()
            torch.cuda.synchronize()
            kt[s].append(e0.elapsed_time(e1) / args.steps)
        print(f"round {r}: " + "  ".join(f"{kt[s][-1]:.3f}" for s in args.settings), flush=True)
    apply("")
    for s in args.settings:
        print(f"kernel [{s}]: median {statistics.median(kt[s]):.3f} ms  min {min(kt[s]):.3f}")


if __name__ == "__main__":
    main()
