"""Multi-GPU SIF / MMB2: one process per GPU, utterances sharded, one all-reduce.

The hot path shards naturally: the weighted averages (a1/a2),
the frame sums and the MMB2 projection (a6-a8) and the PC removal (a4) are
independent per utterance.  The one exchange is the PC (a3), which the
reference computes from ALL utterances of a split: each rank reduces its
contiguous utterance range [row0, row0+n) to a 300x300 fp64 Gram (plus, in
sklearn's transposed branch for splits smaller than 300 utterances, the
d x k block X^T Omega), one `dist.all_reduce` (RCCL over xGMI; 720 KB, latency
bound) sums them, and every rank solves the identical PC — no broadcast.

Launch with torch.distributed.run (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1); backend "nccl" is RCCL on ROCm, "gloo" runs the same
orchestration on CPU for tests.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

import pipeline as P


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced utterance range (row0, n) of `rank`."""
    base, rem = divmod(n_total, world)
    row0 = rank * base + min(rank, rem)
    return row0, base + (1 if rank < rem else 0)


def init(backend: str | None = None, force_group: bool = False):
    """Initialise the default process group from the torchrun environment.
    Returns (rank, world, device).  A world of one rank gets no group unless
    `force_group` (tests: RCCL itself exercised on one GPU)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if (world > 1 or force_group) and not dist.is_initialized():
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    return rank, world, dev


def allreduce_sum(group=None, force: bool = False):
    """In-place SUM all-reduce of one tensor.  None (nothing to reduce)
    without a process group or with one rank, unless `force`: then the
    collective runs even at world size 1 (tests put RCCL on the step's path)."""
    if not dist.is_available() or not dist.is_initialized():
        return None
    if dist.get_world_size(group) == 1 and not force:
        return None

    def _ar(t: torch.Tensor):
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)

    return _ar


def sharded_pc(num, cnt, npc: int, n_total: int, row0: int, group=None, ops=P.DeviceOps):
    """The global PC of a split from this rank's rows (see pipeline.global_pc)."""
    return P.global_pc(num, cnt, npc, n_total, row0, allreduce_sum(group), ops=ops)


def sharded_sif_embeddings(table, ids_local, wtab32, n_total: int, row0: int, npc: int = 1,
                           out_dtype=torch.float32, group=None):
    """SIF embeddings (a1-a5) of this rank's utterances, PC over all ranks."""
    return P.sif_embeddings(table, ids_local, wtab32=wtab32, npc=npc, out_dtype=out_dtype,
                            allreduce=allreduce_sum(group), n_total=n_total, row0=row0)


def sharded_fused_step(inputs_local: dict, networks: dict, n_total: int, row0: int,
                       npc: int = 1, group=None, allreduce=None) -> P.FusedStep:
    """The bench step on this rank's shard (SIF + MMB2 of every local
    utterance).  Checked: every run() ends with FusedStep.check(), whose flag
    bits are summed over the ranks, so an id >= V (IndexError, like numpy's
    fancy index at sif_functions.py:55) or an all-zero-weight utterance
    (ValueError, TruncatedSVD's input check) on ANY rank raises on every rank.
    `allreduce` overrides the RCCL sum (tests: a fake all-reduce)."""
    return P.FusedStep(inputs_local, networks, npc=npc,
                       allreduce=allreduce if allreduce is not None else allreduce_sum(group),
                       n_total=n_total, row0=row0, check_each_run=True)
