#!/usr/bin/env python3
"""Per-workgroup timeline of the fused stream + projection kernel (tools build).

    python tools/fused_balance.py [--utts 125000 1000000] [--reps 3]

Runs mmb_mm2_stream_project on the configs[3] workload (synth.device_shard)
with the tools build's wall-clock marks (mmb_diag_fused_probe: start, every
streamer / projector wave's end per workgroup) and prints, per size, how the
workgroups' finishing times spread: the end-of-kernel imbalance a dynamic
batch schedule could recover.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG_LIB = os.environ.get("MMB_TOOLS_LIB", os.path.join(ROOT, "tools", "diag", "libmmb_diag.so"))
sys.path.insert(0, os.path.join(ROOT, "multimodal-baselines_amd"))
import mmb_lib  # noqa: E402

mmb_lib.load(DIAG_LIB)  # the tools build: explicit, never through the product loader

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mmb_lib as L  # noqa: E402
import models  # noqa: E402
import pipeline as P  # noqa: E402
import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--utts", type=int, nargs="+", default=[125_000, 1_000_000])
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = L.require_gpu()
    lib = L.load()
    fn = lib.mmb_diag_fused_probe
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    buf = np.zeros(1024 * 9, dtype=np.uint64)
    rate = ctypes.c_int(0)
    for U in args.utts:
        inp = synth.device_shard(0, U, 40, 400_000, seed=1000, device=dev)
        torch.manual_seed(0)
        gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
        step = P.FusedStep(inp, gen.networks())
        for rep in range(args.reps + 1):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            P.mm2_stream_project(step.n, step.t, step.d, step.a, step.vd, inp["audio"], inp["visual"],
                                 step.proj, ids32=step.ids, table=step.table, wtab32=inp["wtab"],
                                 flag=step.flag, out=(step.x, step.aux, step.mmb2),
                                 colmax=step.colmax, colmax_ws=step.colmax_ws)
            b.record()
            torch.cuda.synchronize()
            if rep == 0:
                continue
            assert fn(buf.ctypes.data, ctypes.byref(rate)) == 0
            G = min(256, L.cu_count(dev))
            t = buf[:G * 9].reshape(G, 9).astype(np.float64) * 1e3 / rate.value  # us
            t0 = t[:, 0].min()
            start = t[:, 0] - t0
            s_end = t[:, 1:5].max(1) - t0
            p_end = t[:, 5:9].max(1) - t0
            end = np.maximum(s_end, p_end)
            print(f"U={U} rep {rep}: kernel {a.elapsed_time(b):.3f} ms | start spread "
                  f"{start.max():.1f} us | streamers end min/med/max {s_end.min() / 1e3:.3f}/"
                  f"{np.median(s_end) / 1e3:.3f}/{s_end.max() / 1e3:.3f} ms | projectors "
                  f"{p_end.min() / 1e3:.3f}/{np.median(p_end) / 1e3:.3f}/{p_end.max() / 1e3:.3f} ms"
                  f" | proj lag med {np.median(p_end - s_end):.1f} us | end - median end "
                  f"{(end.max() - np.median(end)):.1f} us | per-XCD (b % 8) median end "
                  + " ".join(f"{np.median(end[x::8]) / 1e3:.3f}" for x in range(8)), flush=True)
        del step, inp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
