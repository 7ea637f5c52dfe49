"""HBM read-rate probes on the bench's audio/visual arrays (linear vs per-utterance order)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multimodal-baselines_amd"))
import torch
import synth

dev = torch.device("cuda", 0)
N, T = 1_000_000, 40
inp = synth.device_workload(N, T, 400_000, seed=1, device=dev)
a, v = inp["audio"], inp["visual"]


def timed(fn, reps=5):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


gb = (a.numel() + v.numel()) * 4 / 1e9
t = timed(lambda: (a.view(-1, 4000).sum(1), v.view(-1, 4000).sum(1)))
print(f"torch linear row-sum of audio+visual ({gb:.1f} GB): {t:.2f} ms = {gb / t:.2f} TB/s")
t = timed(lambda: (a.sum(1), v.sum(1)))
print(f"torch sum over frames [N,T,F]->[N,F]: {t:.2f} ms = {gb / t:.2f} TB/s")
out = torch.empty_like(a[:, 0, :])
t = timed(lambda: torch.sum(a, dim=1, out=out))
print(f"audio only sum(1): {t:.2f} ms = {gb / 2 / t:.2f} TB/s")
