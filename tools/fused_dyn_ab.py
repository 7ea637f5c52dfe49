#!/usr/bin/env python3
"""Same-process A/B of the fused stream + projection kernel's batch order
(tools build, r05): the static round robin (MMB_FUSED_DYN=0) against the
dynamic schedule (each workgroup's streamers draw their next 48-row batch
from a counter).  The bench step at each --n, `--steps` steps per variant
alternated over rounds; per variant the median fused-kernel and step times
(HIP events), and whether the two orders give bit-identical rows.

    python tools/fused_dyn_ab.py [--n 1000000 125000] [--steps 4] [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
import mmb_lib  # noqa: E402

mmb_lib.load(os.path.join(ROOT, "tools", "diag", "libmmb_diag.so"))
import torch  # noqa: E402

import models  # noqa: E402
import pipeline as P  # noqa: E402
import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[1_000_000, 125_000])
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for n in args.n:
        inp = synth.device_shard(0, n, 40, 400_000, seed=1000, device=dev)
        torch.manual_seed(0)
        gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
        st = P.FusedStep(inp, gen.networks())
        res = {"static": {"fused": [], "step": []}, "dynamic": {"fused": [], "step": []}}
        outs = {}
        for _ in range(args.rounds):
            for name in res:
                os.environ["MMB_FUSED_DYN"] = "0" if name == "static" else "1"
                st.run()
                torch.cuda.synchronize()
                for _ in range(args.steps):
                    tr = {}
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    st.run(trace=tr)
                    b.record()
                    torch.cuda.synchronize()
                    res[name]["fused"].append(sum(x.elapsed_time(y) for x, y in tr["mm2_stream_project"]))
                    res[name]["step"].append(a.elapsed_time(b))
                st.check()
                outs[name] = [t.clone() for t in (st.x, st.mmb2, st.sif)]
        os.environ.pop("MMB_FUSED_DYN", None)
        same = all(torch.equal(u, v) for u, v in zip(outs["static"], outs["dynamic"]))
        out = {k: {m: round(statistics.median(v), 4) for m, v in d.items()} for k, d in res.items()}
        print(json.dumps({"n": n, **out, "bit_identical": same}), flush=True)
        del st, inp, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
