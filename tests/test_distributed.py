"""CPU, world_size 2 under gloo: the sharded PC orchestration of distributed.py.

Each rank owns a contiguous utterance range, reduces it to its Gram (and, in
the transposed branch, X^T Omega for ITS rows), one all-reduce sums them, and
both ranks must solve the identical PC that one process gets from all rows —
which is also the reference's PC (golden fixtures).  Kernel calls are
replaced by the oracle's CPU doubles (oracle.sif_oracle.CPUOps); the
partitioning, Omega row slicing and collectives are the product code.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import distributed as D
import pipeline as P
import synth
from oracle import sif_oracle as O


def test_shard_range_partitions():
    for n in (1, 7, 320, 1000, 1_000_003):
        for w in (1, 2, 3, 8):
            parts = [D.shard_range(n, w, r) for r in range(w)]
            assert parts[0][0] == 0
            assert sum(p[1] for p in parts) == n
            for (a0, an), (b0, _) in zip(parts, parts[1:]):
                assert a0 + an == b0
            assert max(p[1] for p in parts) - min(p[1] for p in parts) <= 1


@pytest.mark.parametrize("case", ["g2_mosi", "g1_pom_valid", "g3_gap"])
def test_gram_solver_restatement_matches_reference(golden, case):
    """The device solver's math (Gram-only randomized SVD) reproduces the
    reference's sklearn PC on CPU — also without a spectral gap (g3)."""
    z = golden(case)
    X = torch.from_numpy(z["emb"].astype(np.float32))
    pc = P.global_pc(X, None, 1, X.shape[0], 0, None, ops=O.CPUOps)
    assert np.abs(pc.numpy() - z["pc"]).max() < 1e-10


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, case_path, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X = np.load(case_path).astype(np.float32)  # the split's a2 rows
    n_total = X.shape[0]
    row0, n = D.shard_range(n_total, world, rank)
    # num/cnt as the stream kernel leaves them: any split with num/cnt == X works
    cnt = torch.from_numpy(np.full(n, 4.0, np.float32))  # power of 2: num/cnt == X exactly
    num = torch.from_numpy(X[row0:row0 + n] * np.float32(4.0))
    pc = D.sharded_pc(num, cnt, 1, n_total, row0, ops=O.CPUOps)
    np.save(out_path.format(rank), pc.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case,world", [("g2_mosi", 2), ("g1_pom_valid", 2), ("g2_mosi", 3)])
def test_sharded_pc_gloo(golden, tmp_path, case, world):
    case_path = str(tmp_path / "emb.npy")
    np.save(case_path, golden(case)["emb"])
    out = str(tmp_path / "pc_{}.npy")
    mp.start_processes(_worker, args=(world, _free_port(), case_path, out), nprocs=world,
                       join=True, start_method="spawn")
    pcs = [np.load(out.format(r)) for r in range(world)]
    for p in pcs[1:]:
        assert np.array_equal(p, pcs[0])  # identical on every rank, no broadcast
    z = golden(case)
    assert np.abs(pcs[0] - z["pc"]).max() < 1e-9


def test_single_process_allreduce_is_noop():
    assert D.allreduce_sum() is None
