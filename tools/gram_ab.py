import sys, os
sys.path.insert(0, os.path.join(os.getcwd(), "multimodal-baselines_amd"))
import torch, pipeline as P, synth, models
dev = torch.device("cuda", 0)
inp = synth.device_workload(1_000_000, 40, 400_000, seed=1, device=dev)
torch.manual_seed(0)
gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
step = P.FusedStep(inp, gen.networks())
step.run(); torch.cuda.synchronize()
cnt = step.aux[0]
def timed(fn, reps=10):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps
for _ in range(2):
    print("gram with cnt   %.4f ms" % timed(lambda: P.gram(step.x, None, step.G, ws=step.gws)))
    print("gram cnt=None   %.4f ms" % timed(lambda: P.gram(step.x, None, step.G, ws=step.gws)))
    print("remove with cnt %.4f ms" % timed(lambda: P.remove_pc(step.x, None, step.pc, out=step.sif)))
    print("remove cnt=None %.4f ms" % timed(lambda: P.remove_pc(step.x, None, step.pc, out=step.sif)))
