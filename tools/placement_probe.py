#!/usr/bin/env python3
"""Does the stream kernel's time depend on where its buffers land in HBM?

Within ONE process: for a few padding sizes, allocate a dummy buffer first
(shifting the physical placement of everything allocated after it), build the
configs[3] workload, time mmb_mm2_stream (HIP events, 5 launches), free all.
The process-to-process spread of DESIGN.md §7 (20.2-22.3 ms) is either
placement (varies here) or something per process (constant here)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-baselines_amd"))
import torch  # noqa: E402

import pipeline as P  # noqa: E402
import synth  # noqa: E402
import models  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    for pad_gb in [0, 3, 7, 0, 11, 5, 0]:
        pad = torch.empty(int(pad_gb * 2**30), dtype=torch.uint8, device=dev) if pad_gb else None
        inp = synth.device_workload(1_000_000, 40, 400_000, seed=1000, device=dev)
        x = torch.empty((1_000_000, 300), device=dev)
        kp = P.mm2_dims(300, 300, 300)[0]
        s = P.s_buffer(1_000_000, kp, True, dev)
        aux = torch.empty((3, 1_000_000), device=dev)
        run = lambda: P.mm2_stream(1_000_000, 40, 300, 300, 300, inp["audio"], inp["visual"],
                                   ids32=inp["ids"], table=inp["table"], wtab32=inp["wtab"],
                                   out=(x, s, aux))
        run()
        ts = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        print(f"pad {pad_gb:2d} GB: stream ms {' '.join(f'{t:.2f}' for t in ts)}  "
              f"audio@{inp['audio'].data_ptr():#x}", flush=True)
        del inp, x, s, aux, pad
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
