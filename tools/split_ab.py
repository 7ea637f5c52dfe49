#!/usr/bin/env python3
"""POM's real splits (g11: 100 x 1089, 203 x 1357 tokens): the stream phase
of the one-workgroup-per-utterance kernel (mmb_mm2_stream) against the split
path (mmb_mm2_stream_split) at several part counts, product library, HIP
events around each launch, median of --reps, alternated rounds.  Prints one
JSON line: ms per variant and the frame-byte rate as a fraction of 8 TB/s.

    python tools/split_ab.py [--reps 30]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mmb_lib as L  # noqa: E402

# --lib PATH: an A/B clone of the product library (tools/ab_libs), loaded
# explicitly before the mirror modules bind to it
_lib = next((sys.argv[i + 1] for i, a in enumerate(sys.argv[:-1]) if a == "--lib"), None)
if _lib:
    L.load(_lib)
import pipeline as P  # noqa: E402
import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--parts", default="0,2,3,4,6,8,12,16")
args = ap.parse_args()
dev = L.require_gpu()
z = np.load(os.path.join(ROOT, "tests", "golden", "g11_pom_splits.npz"), allow_pickle=False)
splits = [synth.to_device(sp, dev) for sp in
          synth.pom_splits(z["valid_ids"], z["test_ids"], z["weights"], int(z["table_seed"]))]
variants = ["one"] + [f"p{p}" for p in args.parts.split(",")]
res = {}
for r in range(3):
    for si, inp in enumerate(splits):
        n, t = inp["ids"].shape
        ws = P.split_ws(n, t, 300, 300, 300, dev, parts=16)
        out = (torch.empty((n, 300), device=dev), P.s_buffer(n, P.mm2_dims(300, 300, 300)[0], True, dev),
               torch.empty((3, n), device=dev))
        for v in variants:
            kw = {} if v == "one" else dict(split=ws, parts=int(v[1:]))
            call = lambda: P.mm2_stream(n, t, 300, 300, 300, inp["audio"], inp["visual"],
                                        ids32=inp["ids"], table=inp["table"], wtab32=inp["wtab"],
                                        out=out, **kw)
            for _ in range(3):
                call()
            # 10 calls captured in a graph: the GPU time per call without
            # the host's launch gaps (two ctypes launches per call)
            g = torch.cuda.CUDAGraph()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                with torch.cuda.graph(g):
                    for _ in range(10):
                        call()
            torch.cuda.synchronize()
            g.replay()
            for _ in range(args.reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                g.replay()
                b.record()
                b.synchronize()
                res.setdefault(f"split{si}_{v}", []).append(a.elapsed_time(b) / 10)
# the read ceiling at these sizes: mmb_probe_read over the split's audio and
# visual buffers (one launch each, nt loads), graph-timed like the variants
sink = torch.zeros(64, dtype=torch.int32, device=dev)
for si, inp in enumerate(splits):
    for blocks in (512, 1024, 2048, 4096):
        def call(inp=inp, blocks=blocks):
            for buf in (inp["audio"], inp["visual"]):
                L.call("mmb_probe_read", L.ptr(buf), buf.numel() * 4, blocks, 1, L.ptr(sink),
                       L.stream_ptr())
        call()
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            with torch.cuda.graph(g):
                for _ in range(10):
                    call()
        torch.cuda.synchronize()
        g.replay()
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            g.replay()
            b.record()
            b.synchronize()
            res.setdefault(f"split{si}_read{blocks}", []).append(a.elapsed_time(b) / 10)
    variants_read = [f"read{b}" for b in (512, 1024, 2048, 4096)]
summary = {"auto_parts": [P.split_parts(*inp["ids"].shape) for inp in splits]}
variants = variants + variants_read
for si, inp in enumerate(splits):
    n, t = inp["ids"].shape
    frame_b = 2 * n * t * 300 * 4
    for v in variants:
        ms = statistics.median(res[f"split{si}_{v}"])
        summary[f"split{si}_{v}_ms"] = round(ms, 4)
        summary[f"split{si}_{v}_frac_frames"] = round(frame_b / (ms * 1e-3) / 8e12, 3)
print(json.dumps(summary), flush=True)
