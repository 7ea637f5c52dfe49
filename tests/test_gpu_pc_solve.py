"""The multi-workgroup PC solve (mmb_pc_solve_mc) after r06's changes against
the CPU oracle (oracle.sif_oracle.pc_from_gram, itself pinned to the
reference's TruncatedSVD by the g3 fixtures, tests/test_oracle_golden.py):

  * squared rounds: one product by G, then (n_iter - 1) / 2 by G2 = G G
    (formed by extra workgroups of the same launch, or by the transposed
    start's prep launch), the rest and the tail by G -- every n_iter 0..8
    (odd and even: the fragment reloads), direct and transposed branches,
    npc = 1 (squared) and npc = 2 (not squared);
  * the direct branch's last round exchanged beside its factor, and a
    rank-deficient block whose Cholesky pivots fail there (MGS^2 fallback,
    a second exchange);
  * the same G and z0 give the same PC bit for bit, eager and graph replay.

Reference: /root/reference/sif_functions.py:58-67 (compute_pc).
"""
import numpy as np
import pytest
import torch

import pipeline as P
from oracle import sif_oracle as O

pytestmark = pytest.mark.gpu


def _case(n, d=300, rank=None, seed=0, scale=0.4):
    g = torch.Generator(device="cpu").manual_seed(seed)
    if rank is None:
        x = scale * torch.randn(n, d, generator=g, dtype=torch.float64)
        x += 0.3 * torch.randn(d, generator=g, dtype=torch.float64)
    else:
        x = torch.randn(n, rank, generator=g, dtype=torch.float64) @ torch.randn(
            rank, d, generator=g, dtype=torch.float64)
    return x


def _solve(x, npc, n_iter, dev):
    n, d = x.shape
    k = npc + P.N_OVERSAMPLES
    G = (x.T @ x).to(dev)
    if n >= d:
        z0, tr = P.omega(d, k, dev).clone(), False
    else:
        z0, tr = (x.T @ P.omega(n, k, "cpu")).to(dev), True
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    pc = P.pc_solve(G, z0, npc, tr, n_iter=n_iter, flag=flag).clone()
    torch.cuda.synchronize()
    assert int(flag.item()) == 0
    ref = O.pc_from_gram(G.cpu().numpy(), z0.cpu().numpy(), npc, tr, n_iter=n_iter)
    return G, z0, tr, pc, ref


@pytest.mark.parametrize("n_iter", [0, 1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("n", [4096, 180])
def test_squared_rounds_every_n_iter(gpu, n, n_iter):
    x = _case(n, seed=n_iter)
    _, _, _, pc, ref = _solve(x, 1, n_iter, gpu)
    assert np.abs(pc.cpu().numpy() - ref).max() < 1e-12


@pytest.mark.parametrize("n", [4096, 180])
def test_npc2_unsquared(gpu, n):
    x = _case(n, seed=11)
    _, _, _, pc, ref = _solve(x, 2, 7, gpu)
    assert np.abs(pc.cpu().numpy() - ref).max() < 1e-10


@pytest.mark.parametrize("n,rank", [(1000, 4), (2000, 9), (150, 3)])
def test_rank_deficient_block_falls_back(gpu, n, rank):
    """rank < k = 11: the block's Gram is singular, every Cholesky pivot past
    the rank fails and the rounds (the direct branch's last one included)
    take the MGS^2 fallback with its second exchange."""
    x = _case(n, rank=rank, seed=rank)
    n_, d = x.shape
    k = 1 + P.N_OVERSAMPLES
    G = (x.T @ x).to(gpu)
    tr = n_ < d
    z0 = (x.T @ P.omega(n_, k, "cpu")).to(gpu) if tr else P.omega(d, k, gpu).clone()
    flag = torch.zeros(1, dtype=torch.int32, device=gpu)
    pc = P.pc_solve(G, z0, 1, tr, flag=flag).cpu().numpy()[0]
    assert int(flag.item()) == 0 and np.isfinite(pc).all()
    # the block spans G's whole range (rank < k): the PC is G's top
    # eigenvector to rounding (the oracle's direct branch factors the
    # singular Z^T G Z and cannot take this case)
    w, v = np.linalg.eigh(G.cpu().numpy())
    top = v[:, -1] * np.sign(v[np.argmax(np.abs(v[:, -1])), -1])
    assert np.abs(pc - top).max() < 1e-9


def test_deterministic_and_graph_replay(gpu):
    x = _case(4096, seed=5)
    G, z0, tr, pc, _ = _solve(x, 1, 7, gpu)
    out = torch.empty_like(pc)
    flag = torch.zeros(1, dtype=torch.int32, device=gpu)
    ws = P.solve_workspace(300, gpu)
    for _ in range(3):
        P.pc_solve(G, z0, 1, tr, out=out, flag=flag, ws=ws)
        torch.cuda.synchronize()
        assert torch.equal(out, pc)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    gws = torch.zeros_like(ws)
    with torch.cuda.stream(side):
        P.pc_solve(G, z0, 1, tr, out=out, flag=flag, ws=gws)  # warm (attributes)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            P.pc_solve(G, z0, 1, tr, out=out, flag=flag, ws=gws)
    for _ in range(4):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, pc) and int(flag.item()) == 0


@pytest.mark.parametrize("n,npc", [(100, 1), (229, 1), (180, 2), (7, 1)])
def test_transposed_start_in_one_launch(gpu, n, npc):
    """mmb_pc_solve_mc_xt (X^T Omega and G2 in one launch, then the solve)
    against mmb_xt_omega + mmb_pc_solve_mc: the same z0 sums, the same PC
    bit for bit; and against the oracle."""
    import mmb_lib as L
    g = torch.Generator(device="cpu").manual_seed(n)
    x = (0.4 * torch.randn(n, 300, generator=g) + 0.3 * torch.randn(300, generator=g)).to(gpu)
    k = npc + P.N_OVERSAMPLES
    G = (x.double().T @ x.double()).contiguous()
    om = P.omega(n, k, gpu)
    z0 = P.xt_omega(x, None, om)
    flag = torch.zeros(1, dtype=torch.int32, device=gpu)
    ref = P.pc_solve(G, z0, npc, True, flag=flag).clone()
    ws = torch.zeros(L.query("mmb_pc_solve_mc_ws_bytes", 300), dtype=torch.uint8, device=gpu)
    pc = torch.empty((npc, 300), dtype=torch.float64, device=gpu)
    L.call("mmb_pc_solve_mc_xt", L.ptr(G), 300, L.ptr(x), n, L.ptr(om), k, npc, P.N_ITER, L.ptr(pc),
           L.ptr(ws), L.ptr(flag), L.stream_ptr())
    torch.cuda.synchronize()
    assert int(flag.item()) == 0 and not bool(ws[:16].any())
    assert torch.equal(pc, ref)
    oracle = O.pc_from_gram(G.cpu().numpy(), z0.cpu().numpy(), npc, True)
    assert np.abs(pc.cpu().numpy() - oracle).max() < 1e-10
