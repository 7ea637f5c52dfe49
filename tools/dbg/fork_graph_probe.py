#!/usr/bin/env python3
"""Which capture pattern of the forked projection survives a concurrent
StepGraph (r06 probe: the two POM steps, each forking its projection, in one
graph with concurrent branches segfaulted in capture_end).  One variant per
process (argv[1]); prints 'ok <variant>' when the graph captures and replays
with rows equal to eager.  Measured (gpurun_out r06probe): a fork joined to
its branch stream -- with torch's temporary events or persistent ones --
segfaulted in capture_end; StepGraph(concurrent=False) and forks joined to
the capture's origin stream (what StepGraph now does) capture and replay.

  concurrent : the product StepGraph (forks joined at the origin stream)
  serial     : StepGraph(concurrent=False) with the forks
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mmb_lib as L  # noqa: E402
import models  # noqa: E402
import pipeline as P  # noqa: E402
import synth  # noqa: E402

v = sys.argv[1]
dev = L.require_gpu()
z = np.load(os.path.join(ROOT, "tests", "golden", "g11_pom_splits.npz"), allow_pickle=False)
splits = synth.pom_splits(z["valid_ids"], z["test_ids"], z["weights"], int(z["table_seed"]))
torch.manual_seed(0)
gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
steps = [P.FusedStep(synth.to_device(sp, dev), gen.networks()) for sp in splits]
eager = [[t.clone() for t in st.run(check=True)] for st in steps]
g = P.StepGraph(steps, concurrent=(v != "serial"))
print("captured", v, flush=True)
for _ in range(2):
    outs = g.run(check=True)
for (s0, m0), (s1, m1) in zip(eager, outs):
    assert torch.equal(s0, s1) and torch.equal(m0, m1)
print("ok", v, flush=True)
