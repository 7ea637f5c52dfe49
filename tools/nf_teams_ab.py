#!/usr/bin/env python3
"""Same-process A/B of the narrow fused kernel's batch organisation (tools
build, r05): one 32-row batch per workgroup with workgroup barriers
(MMB_NF_TEAMS=0, the product) against two teams of 4 waves running 16-row
batches on their own LDS halves with their own barriers (1), and the same
with team 1 starting one stream phase later (2).  The MOSI bench step at each
--n, `--steps` steps per variant alternated over rounds; per variant the
median kernel and step times (HIP events), and whether the variants' rows
are bit-identical to the product's.

    python tools/nf_teams_ab.py [--n 1000000 1284] [--steps 4] [--rounds 3]
    python tools/nf_teams_ab.py --knob NAME --values V0 V1 ...   (another narrow-kernel knob;
        r05's utterance-pair knob MMB_NF_ILP was measured this way, profiles/r05_narrow/pairs_ab.txt,
        and removed)
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
import mmb_lib  # noqa: E402

# (MMB_TOOLS_LIB: another tools-build library, e.g. one with other NF_* build knobs)
mmb_lib.load(os.environ.get("MMB_TOOLS_LIB", os.path.join(ROOT, "tools", "diag", "libmmb_diag.so")))
import torch  # noqa: E402

import models  # noqa: E402
import pipeline as P  # noqa: E402
import synth  # noqa: E402

VARIANTS = {"one_batch": "0", "teams": "1", "teams_lag": "2"}
KNOB = "MMB_NF_TEAMS"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[1_000_000, 1284])
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", nargs="+", default=list(VARIANTS))
    ap.add_argument("--knob", default=None, help="another tools-build knob, with "
                                                 "--values (variant name = value)")
    ap.add_argument("--values", nargs="+", default=None)
    args = ap.parse_args()
    global KNOB
    if args.knob:
        KNOB = args.knob
        VARIANTS.clear()
        VARIANTS.update({f"{args.knob}={v}": v for v in args.values})
        args.variants = list(VARIANTS)
    dev = torch.device("cuda", 0)
    T, V, A, Vd = 20, 3016, 76, 48
    for n in args.n:
        inp = synth.device_workload(n, T, V, D=300, A=A, Vd=Vd, seed=4000, device=dev)
        torch.manual_seed(0)
        gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(dev)
        st = P.FusedStep(inp, gen.networks(), narrow_fused=True)
        res = {k: {"kernel": [], "step": []} for k in args.variants}
        outs = {}
        for _ in range(args.rounds):
            for name in args.variants:
                os.environ[KNOB] = VARIANTS[name]
                st.run()
                torch.cuda.synchronize()
                for _ in range(args.steps):
                    tr = {}
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    st.run(trace=tr)
                    b.record()
                    torch.cuda.synchronize()
                    res[name]["kernel"].append(sum(x.elapsed_time(y) for x, y in tr["mm2_stream_project_narrow"]))
                    res[name]["step"].append(a.elapsed_time(b))
                st.check()
                outs[name] = [t.clone() for t in (st.x, st.mmb2, st.sif)]
        os.environ.pop(KNOB, None)
        base = outs[args.variants[0]]
        same = {k: all(torch.equal(u, v) for u, v in zip(base, o)) for k, o in outs.items()}
        out = {k: {m: round(statistics.median(v), 4) for m, v in d.items()} for k, d in res.items()}
        print(json.dumps({"n": n, **out, "bit_identical": same}), flush=True)
        del st, inp, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
