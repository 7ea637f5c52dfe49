#!/usr/bin/env python3
"""Eager FusedStep launches against one HIP-graph replay of the same step
(StepGraph) at the bench shapes (r05): wall time of `steps` steps between two
device syncs, alternated over rounds; the median per step of each, the host
time to enqueue them (*_host_enqueue: the host runs ahead of the device when
it is well below the step), and the rows of the two compared bit for bit.

    python tools/graph_step_ab.py [--n 125000 1000000] [--steps 20] [--rounds 3] [--mosi]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
import torch  # noqa: E402

import models  # noqa: E402
import pipeline as P  # noqa: E402
import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[125_000, 1_000_000])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--mosi", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for n in args.n:
        if args.mosi:
            A = Vd = None
            inp = synth.device_workload(n, 20, 3016, D=300, A=76, Vd=48, seed=4000, device=dev)
            A, Vd = 76, 48
        else:
            A = Vd = 300
            inp = synth.device_shard(0, n, 40, 400_000, seed=1000, device=dev)
        torch.manual_seed(0)
        gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(dev)
        st = P.FusedStep(inp, gen.networks())
        for _ in range(3):
            st.run()
        torch.cuda.synchronize()
        st.check()
        eager_rows = [t.clone() for t in (st.sif, st.mmb2)]
        g = P.StepGraph(st)
        g.run(check=True)
        same = all(torch.equal(u, v) for u, v in zip(eager_rows, (st.sif, st.mmb2)))
        res = {"eager": [], "graph": []}
        for _ in range(args.rounds):
            for name in ("eager", "graph"):
                f = st.run if name == "eager" else g.run
                f()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    f()
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                res[name].append((time.perf_counter() - t0) * 1e3 / args.steps)
                res.setdefault(name + "_host_enqueue", []).append((t1 - t0) * 1e3 / args.steps)
        st.check()
        print(json.dumps({"n": n, "mosi": args.mosi,
                          **{k: round(statistics.median(v), 4) for k, v in res.items()},
                          "all": {k: [round(x, 4) for x in v] for k, v in res.items()},
                          "graph_rows_equal_eager": same}), flush=True)
        del g, st, inp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
