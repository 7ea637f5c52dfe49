#!/usr/bin/env python3
"""Which buffer's placement moves the stream kernel?  One workload; then
re-place one input at a time (clone it behind a fresh padding allocation,
free the old copy) and time mmb_mm2_stream after each move."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-baselines_amd"))
import torch  # noqa: E402

import pipeline as P  # noqa: E402
import synth  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    inp = synth.device_workload(1_000_000, 40, 400_000, seed=1000, device=dev)
    x = torch.empty((1_000_000, 300), device=dev)
    kp = P.mm2_dims(300, 300, 300)[0]
    s = P.s_buffer(1_000_000, kp, True, dev)
    aux = torch.empty((3, 1_000_000), device=dev)

    def timed():
        x, s, aux = outs["x"], outs["s"], outs["aux"]
        run = lambda: P.mm2_stream(1_000_000, 40, 300, 300, 300, inp["audio"], inp["visual"],
                                   ids32=inp["ids"], table=inp["table"], wtab32=inp["wtab"],
                                   out=(x, s, aux))
        run()
        ts = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            run()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return " ".join(f"{t:.2f}" for t in ts)

    outs = {"x": x, "s": s, "aux": aux}
    print("start:", timed(), flush=True)
    pads = []
    outs = {"x": x, "s": s, "aux": aux}
    for it, key in enumerate(["s", "s", "s", "x", "x", "x", "s", "visual", "audio", "s", "x"]):
        pads.append(torch.empty(int((it % 4 + 1) * 2**29), dtype=torch.uint8, device=dev))
        src = outs if key in outs else inp
        new = src[key].clone()
        del src[key]
        torch.cuda.empty_cache()
        src[key] = new
        x, s, aux = outs["x"], outs["s"], outs["aux"]
        print(f"moved {key:6s}:", timed(), flush=True)


if __name__ == "__main__":
    main()
