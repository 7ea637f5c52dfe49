#!/usr/bin/env python3
"""Timing of one build of the narrow fused kernel (mmb_mm2_stream_project_narrow)
on the MOSI bench workload (1M utterances, T 20, A 76, Vd 48, V 3016): the
kernel's mean launch time over --steps FusedStep runs, the step time, and the
a2 rows against the two-kernel step's (row-relative).  One library per
process (tools/ab_libs/build_nf.sh builds the knob variants):

    python tools/nf_ab.py --lib tools/ab_libs/libmmb_nf_4_1.so
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-baselines_amd"))
sys.path.insert(0, ROOT)
import mmb_lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", required=True)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--workload", choices=["mosi", "synthetic"], default="mosi",
                    help="synthetic: the headline configs[3] step (T 40, 3 x 300-d, V 400k)")
    args = ap.parse_args()
    # the launched instantiation must be in the library's code object: HIP
    # aborts the process otherwise (r05: libmmb_nf_w12_2_1_4_2.so)
    import re
    sys.path.insert(0, os.path.join(ROOT, "tools", "ab_libs"))
    import symcheck
    name = os.path.basename(args.lib)
    m = re.match(r"libmmb_nf_w(\d+)_(\d+)_(\d+)_(\d+)_(\d+)", name)
    want = (symcheck.narrow_symbol(*map(int, m.groups()[1:])) if m else None)
    if want and want not in symcheck.device_symbols(os.path.abspath(args.lib)):
        print(f"{name}: {want} not in its gfx950 code object; not loaded", flush=True)
        return 2
    mmb_lib.load(os.path.abspath(args.lib))
    import torch
    import models
    import pipeline as P
    import synth
    dev = torch.device("cuda:0")
    if args.workload == "mosi":
        T, V, A, Vd = 20, 3016, 76, 48
        inp = synth.device_workload(args.n, T, V, D=300, A=A, Vd=Vd, seed=4000, device=dev)
    else:
        T, V, A, Vd = 40, 400_000, 300, 300
        inp = synth.device_shard(0, args.n, T, V, D=300, A=A, Vd=Vd, seed=1000, device=dev)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(dev)
    step = P.FusedStep(inp, gen.networks(), narrow_fused=args.workload == "mosi")
    for _ in range(3):
        step.run()
    torch.cuda.synchronize()
    traces = [dict() for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step.run(trace=traces[k])
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / args.steps
    try:
        step.check()
    except Exception as e:  # timing-only ablations (NF_ABL) compute no valid step
        print(f"# {os.path.basename(args.lib)} check: {type(e).__name__}", flush=True)
    kn = "mm2_stream_project_narrow" if args.workload == "mosi" else "mm2_stream_project"
    kms = sum(a.elapsed_time(b) for tr in traces for a, b in tr.get(kn, ())) / args.steps
    line = f"{os.path.basename(args.lib)} kernel_ms {kms:.4f} step_ms {ms:.4f}"
    if args.check:
        b = P.FusedStep(inp, gen.networks(), narrow_fused=False, stream_project=False)
        b.run(check=True)
        torch.cuda.synchronize()
        dx = ((step.x - b.x).abs().amax(1) / b.x.abs().amax(1).clamp_min(1e-30)).max().item()
        dm = ((step.mmb2 - b.mmb2).abs().amax(1) / b.mmb2.abs().amax(1).clamp_min(1e-30)).max().item()
        line += f" x_row_rel {dx:.2e} mmb2_row_rel {dm:.2e}"
    print(line, flush=True)


if __name__ == "__main__":
    sys.exit(main())
