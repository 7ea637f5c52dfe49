"""Debug: is the PC solve (mmb_pc_solve_mc) stable across HIP-graph replays?"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
import numpy as np
import torch
import mmb_lib as L, models, pipeline as P, synth

dev = torch.device("cuda", 0)
torch.manual_seed(0)
X = torch.randn(2000, 300, device=dev, dtype=torch.float64) * 0.4 + 0.3 * torch.randn(300, device=dev, dtype=torch.float64)
G = X.T @ X
z0 = P.omega(300, 11, dev)
flag = torch.zeros(1, dtype=torch.int32, device=dev)
ws = torch.zeros(L.query("mmb_pc_solve_mc_ws_bytes", 300), dtype=torch.uint8, device=dev)
pc = torch.empty((1, 300), dtype=torch.float64, device=dev)
P.pc_solve(G, z0, 1, False, out=pc, flag=flag, ws=ws)
torch.cuda.synchronize()
ref = pc.clone()
for mode in ("mc", "single"):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        P.pc_solve(G, z0, 1, False, out=pc, flag=flag, ws=ws) if mode == "mc" else \
            L.call("mmb_pc_solve", L.ptr(G), 300, L.ptr(z0), 11, 1, 7, 0, L.ptr(pc), L.stream_ptr())
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        if mode == "mc":
            P.pc_solve(G, z0, 1, False, out=pc, flag=flag, ws=ws)
        else:
            L.call("mmb_pc_solve", L.ptr(G), 300, L.ptr(z0), 11, 1, 7, 0, L.ptr(pc), L.stream_ptr())
    for r in range(4):
        pc.zero_()
        g.replay()
        torch.cuda.synchronize()
        print(mode, "replay", r, "flag", int(flag.item()), "maxdiff", float((pc - ref).abs().max()),
              "ctl", ws[:8].view(torch.int32).tolist(), flush=True)
    # eager after the graph
    P.pc_solve(G, z0, 1, False, out=pc, flag=flag, ws=ws)
    torch.cuda.synchronize()
    print(mode, "eager after", float((pc - ref).abs().max()), flush=True)
