"""bench.py's world > 1 branch on the GPU box: two ranks sharing GPU 0.

The driver's scaling runs launch `bench.py --gpus N` on an 8-GPU node with
RCCL; a one-GPU box cannot host N RCCL ranks, so this test runs the same
branch -- self-launch through torch.distributed.run, process-group init,
barriers, the per-step Gram all-reduce, the MAX-over-ranks timing, check()'s
flag all-reduce, the rank != 0 early exit and rank 0's JSON line -- with the
collectives on gloo and both ranks on GPU 0 (`--dist-backend gloo
--share-device`), as a fresh child process.  Each rank dumps its PC and a
sample of its rows; they must equal the unsharded step over the same split
(synth.device_shard rebuilds the union of the shards in this process): the
PC within 1e-10, MMB2 rows bit for bit (they never cross ranks), SIF rows to
the removal's dot order.  The reference is single-device
(/root/reference/simplesif.py:243-249); the one global PC per split it
implies (:296-299) is what the all-reduce preserves.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import models
import pipeline as P
import synth
from oracle import mmb2_oracle as M

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("utts,ranks", [(200_000, 2), (90_001, 3)])
def test_bench_multi_rank_branch_matches_unsharded(gpu, tmp_path, utts, ranks):
    V = 50_000
    dump = str(tmp_path / "dump")
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(ranks),
           "--dist-backend", "gloo", "--share-device", "--utts", str(utts), "--vocab", str(V),
           "--steps", "2", "--warmup", "1", "--only-main", "--no-cpu-baseline",
           "--dump-rows", dump]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == ranks and line["ranks_seen"] == ranks
    assert line["scaling"] == "strong" and line["config"]["utts_total"] == utts
    assert line["phase_ms"].get("allreduce") is not None
    assert line["value"] > 0 and line["ms_per_step"] > 0

    inp = synth.device_shard(0, utts, 40, V, seed=1000, device=gpu)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(gpu)
    whole = P.FusedStep(inp, gen.networks())
    s_ref, m_ref = whole.run(check=True)
    pc_ref = whole.pc.cpu().numpy()
    seen = 0
    for rank in range(ranks):
        z = np.load(os.path.join(dump, f"rank{rank}.npz"))
        row0, n = int(z["row0"]), int(z["n"])
        assert row0 == seen
        seen += n
        assert int(z["flag"]) == 0
        assert np.abs(z["pc"] - pc_ref).max() < 1e-10, rank
        rows = torch.as_tensor(row0 + z["idx"], device=gpu)
        assert np.array_equal(z["mmb2"], m_ref[rows].cpu().numpy()), rank
        assert M.row_rel_err(z["sif"], s_ref[rows].cpu().numpy()) < 1e-6, rank
    assert seen == utts
