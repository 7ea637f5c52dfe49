"""Debug (r05): the cause of the r04e dataset_splits failure.

r04e's bench leg raised check_pc_finite's ValueError on a HIP-graph replay of
a split step (gpurun_out/r04e/splits.err) with the library of ae7b7c5, whose
mmb_pc_solve_mc enqueued a 16-byte hipMemsetAsync of its control words
(arrival counter, abort word) before every launch.  This replays the bench's
split flow with a given library and, after every replay, prints the control
words of every split's solve workspace, the flag and whether the PC is
finite -- so a failure shows which word was wrong and with what value:
  abort word == 1        set by a workgroup that timed out (then the flag has
                         MMB_FLAG_SYNC_TIMEOUT too)
  abort word other != 0  written by something else ("garbage")
  counter != 0 before    a stale count (waits pass early)

    [DBG_PKG=tools/dbg/_prefix_pkg] python tools/dbg/replay_cause.py [replays]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
# DBG_PKG: another tree's package directory (its Python mirror and its own
# libmmb.so), e.g. the pre-fix tree copied to tools/dbg/_prefix_pkg
if os.environ.get("DBG_PKG"):
    sys.path.insert(0, os.path.abspath(os.environ["DBG_PKG"]))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mmb_lib as L  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
L.load()
import models  # noqa: E402
import pipeline as P  # noqa: E402
import synth  # noqa: E402

dev = torch.device("cuda", 0)
print("library", L.loaded_path(), "pipeline", P.__file__, flush=True)


def words(st):
    w = st.solve_ws[:16].view(torch.int32).cpu().tolist()
    return w[:2]


def show(tag, steps):
    torch.cuda.synchronize()
    out = []
    for i, st in enumerate(steps):
        out.append(f"s{i}: flag {int(st.flag.item())} ctl {words(st)} "
                   f"pc_finite {bool(torch.isfinite(st.pc).all())}")
    print(tag, " | ".join(out), flush=True)
    return all(bool(torch.isfinite(st.pc).all()) for st in steps)


# 1. the solve alone in a graph, replayed with the same inputs
torch.manual_seed(0)
X = torch.randn(2000, 300, device=dev, dtype=torch.float64) * 0.4
G = X.T @ X
z0 = P.omega(300, 11, dev)
flag = torch.zeros(1, dtype=torch.int32, device=dev)
ws = torch.zeros(L.query("mmb_pc_solve_mc_ws_bytes", 300), dtype=torch.uint8, device=dev)
pc = torch.empty((1, 300), dtype=torch.float64, device=dev)
P.pc_solve(G, z0, 1, False, out=pc, flag=flag, ws=ws)
torch.cuda.synchronize()
ref = pc.clone()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    P.pc_solve(G, z0, 1, False, out=pc, flag=flag, ws=ws)
bad = 0
for r in range(reps):
    pc.zero_()
    g.replay()
    torch.cuda.synchronize()
    w = ws[:16].view(torch.int32).cpu().tolist()
    ok = bool(torch.equal(pc, ref))
    if not ok or r < 3 or w[:2] != [w[0], 0]:
        print(f"solve replay {r}: flag {int(flag.item())} ctl {w[:4]} pc_equal {ok} "
              f"pc_finite {bool(torch.isfinite(pc).all())}", flush=True)
    bad += not ok
print(f"solve alone: {bad} of {reps} replays wrong", flush=True)
del g

# 2. the bench's dataset_splits flow (MOSI: three splits, POM: two)
z = np.load(os.path.join(ROOT, "tests", "golden", "g11_pom_splits.npz"), allow_pickle=False)
sets = {"mosi": (synth.mosi_splits(), 76, 48),
        "pom": (synth.pom_splits(z["valid_ids"], z["test_ids"], z["weights"],
                                 int(z["table_seed"])), 300, 300)}
for name, (splits, A, Vd) in sets.items():
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(dev)
    steps = [P.FusedStep(synth.to_device(sp, dev), gen.networks()) for sp in splits]
    for i, st in enumerate(steps):
        st.run(check=True)
        for _ in range(3):
            st.run(check=True)
        show(f"{name} split {i} eager", [st])
        gr = P.StepGraph(st)
        show(f"{name} split {i} after capture", [st])
        for r in range(reps):
            gr.graph.replay()
            if not show(f"{name} split {i} replay {r}", [st]) and r > 8:
                break
            st.reset()
        del gr
    gall = P.StepGraph(steps, concurrent=True)
    for r in range(reps):
        gall.graph.replay()
        if not show(f"{name} all-splits replay {r}", steps) and r > 8:
            break
        for st in steps:
            st.reset()
    del gall
print("done", flush=True)
