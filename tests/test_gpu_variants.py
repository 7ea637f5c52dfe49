"""Measured kernel variants against the product defaults (tools build).

The product library carries only the default kernels and reads no
environment variable (`strings libmmb.so` has no MMB_* knob); the variants
and timing-only ablations live in tools/diag/libmmb_diag.so (`make diag`;
__graft_entry__.build() makes it beside libmmb.so and it travels to the GPU
box with the tree -- a missing tools build FAILS these tests rather than
skipping them, so the timeout path is part of every GPU run).  Each group
of tests/variant_checks.py runs in ONE child process that loads that build
explicitly; the fused-streamer group also dumps the group-at-a-time
streamer's outputs, which the product library (this process) must reproduce
bit for bit with its default streamer.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import mmb_lib as L
import variant_checks as VC

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG = VC.DIAG_LIB
pytestmark = pytest.mark.gpu


def _child(group, tmp_path):
    assert os.path.exists(DIAG), ("tools build absent: make -C multimodal-baselines_amd/csrc diag "
                                  "(__graft_entry__.build() makes it)")
    env = {**os.environ, "VARIANT_DUMP": str(tmp_path)}
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "variant_checks.py"),
                        group], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


@pytest.mark.parametrize("group", ["projection", "fused_order", "remove_rows", "gram", "narrow_teams",
                                   "timeouts"])
def test_variants_agree(gpu, tmp_path, group):
    _child(group, tmp_path)


def test_fused_streamers_and_product_default(gpu, tmp_path):
    """Streamer / tail variants bit-identical in the tools build, and the
    product library's default launch bit-identical to the group-at-a-time
    streamer on every case (pipe 2 + balanced tail where rows have >= 3 frame
    groups, the group-at-a-time fallback below)."""
    _child("fused_streamer", tmp_path)
    names = ["x", "aux", "mmb2", "colmax", "flag"]
    for ci, (N, T, A, Vd, dense, bad) in enumerate(VC.FUSED_CASES):
        inp, proj = VC.fused_case(gpu, N, T, A, Vd, bad)
        got = VC.fused_outputs(inp, proj, N, T, A, Vd, dense=dense)
        ref = np.load(str(tmp_path / f"fused_{ci}.npz"))
        for nm, g in zip(names, got):
            r = torch.from_numpy(ref[nm]).to(gpu)
            assert torch.equal(torch.nan_to_num(r, nan=7.0), torch.nan_to_num(g, nan=7.0)), (nm, ci)
