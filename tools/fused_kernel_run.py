#!/usr/bin/env python3
"""Launch one kernel of the bench workload R times (for rocprofv3 PMC passes):
the fused stream + projection kernel (MMB_FUSED_DIAG ablations via --diag)
or the plain stream kernel.

    python tools/fused_kernel_run.py {fused,stream} [--diag D] [--reps R] [--n N]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", choices=["fused", "stream"])
    ap.add_argument("--diag", default="0")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n", type=int, default=1_000_000)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    inp = synth.device_workload(args.n, 40, 400_000, seed=1, device=dev)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
    st = P.FusedStep(inp, gen.networks(), stream_project=args.which == "fused")
    kw = dict(audio=inp["audio"], visual=inp["visual"], ids32=inp["ids"], table=inp["table"],
              wtab32=inp["wtab"], colmax=st.colmax, colmax_ws=st.colmax_ws)
    os.environ["MMB_FUSED_DIAG"] = args.diag
    for _ in range(args.reps):
        if args.which == "fused":
            P.mm2_stream_project(st.n, 40, 300, 300, 300, proj=st.proj, out=(st.x, st.aux, st.mmb2), **kw)
        else:
            P.mm2_stream(st.n, 40, 300, 300, 300, out=(st.x, st.s, st.aux), **kw)
    torch.cuda.synchronize()
    print("done", args.which, args.diag)


if __name__ == "__main__":
    main()
