"""Debug: per-split StepGraph replays after eager runs (bench dataset_splits flow)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
import numpy as np
import torch
import models, pipeline as P, synth

dev = torch.device("cuda", 0)
z = np.load(os.path.join(ROOT, "tests", "golden", "g11_pom_splits.npz"))
sets = {"mosi": (synth.mosi_splits(), 76, 48),
        "pom": (synth.pom_splits(z["valid_ids"], z["test_ids"], z["weights"], int(z["table_seed"])), 300, 300)}
for name, (splits, A, Vd) in sets.items():
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(dev)
    steps = [P.FusedStep(synth.to_device(sp, dev), gen.networks()) for sp in splits]
    for i, st in enumerate(steps):
        st.run(check=True)
        pc0 = st.pc.clone()
        for _ in range(5):
            st.run(check=True)
        g = P.StepGraph(st)
        for r in range(3):
            g.run()
            torch.cuda.synchronize()
            print(name, i, "replay", r, "flag", int(st.flag.item()), "pc finite", bool(torch.isfinite(st.pc).all()),
                  "G finite", bool(torch.isfinite(st.G).all()), "pc eq", bool(torch.equal(st.pc, pc0)),
                  "stream_project", st.stream_project, "gram_i8", st.gram_i8, "fused_remove", st.fused_remove, flush=True)
