"""Drop-in for `/root/reference/sif_functions.py` — same names, arguments, dtypes.

Inputs and outputs are numpy arrays exactly as in the reference; the
arithmetic runs on the GPU through libmmb (no CPU fallback):

* seq2weight            -> mmb_seq2weight   (bit-exact, sif_functions.py:8-15)
* get_weighted_average  -> mmb_sif_wavg     (fp32 rows, f64 result, :28-56)
* compute_pc            -> mmb_gram + mmb_pc_solve (sklearn TruncatedSVD(npc,
                           n_iter=7, random_state=0) replayed on the Gram, :58-67)
* remove_pc             -> the above + mmb_pc_remove (f64, :69-81)
* SIF_embedding         -> all of it fused on device, one upload/download (:84-96)

Numerics: rows are reduced in fp32 like the reference's f32 sgemv (an f64 word
table is rounded to f32 first).  compute_pc / remove_pc take X as given: when X
is f32-representable (what get_weighted_average produces) it enters the f32-row
kernels exactly; any other float64 X takes the f64-row kernels (mmb_gram_f64,
mmb_pc_remove_f64), so it is never rounded.  The Gram, the solve and the
removal are fp64.  Non-finite X raises ValueError like sklearn's check_array in
the reference's TruncatedSVD.
"""
from __future__ import annotations

import numpy as np
import torch

import mmb_lib as L
import pipeline as P


class Params(object):
    """sif_functions.py:17-26."""

    def __init__(self):
        self.LW = 1e-5
        self.LC = 1e-5
        self.eta = 0.05

    def __str__(self):
        t = "LW", self.LW, ", LC", self.LC, ", eta", self.eta
        return " ".join(map(str, t))


def _dev():
    return L.require_gpu()


def _ids(x, dev):
    x = np.asarray(x)
    if x.dtype.kind not in "iu":
        raise IndexError("arrays used as indices must be of integer type")
    return P.narrow_ids(torch.from_numpy(np.ascontiguousarray(x.astype(np.int64, copy=False))).to(dev))


def seq2weight(seq, mask, weight4ind):
    """w[i,j] = weight4ind[seq[i,j]] where mask > 0 and seq >= 0, as float32."""
    dev = _dev()
    seq = np.asarray(seq)
    ids = _ids(seq, dev)
    sel = torch.from_numpy(np.ascontiguousarray(np.asarray(mask) > 0).astype(np.uint8)).to(dev)
    wt = torch.from_numpy(np.ascontiguousarray(np.asarray(weight4ind, dtype=np.float64))).to(dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    w = P.seq2weight(ids, sel, wt, flag)
    P.check_flag(flag, wt.numel())
    return w.cpu().numpy()


def _table(We, dev):
    return torch.as_tensor(np.ascontiguousarray(np.asarray(We, dtype=np.float32))).to(dev)


def get_weighted_average(We, x, w):
    """emb[i] = w[i].dot(We[x[i]]) / count_nonzero(w[i])  -> float64 [N, D]."""
    dev = _dev()
    table = _table(We, dev)
    ids = _ids(x, dev)
    wt = torch.as_tensor(np.ascontiguousarray(np.asarray(w, dtype=np.float32))).to(dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    emb = P.weighted_sum(table, ids, w=wt, flag=flag, x_out=True)
    P.check_flag(flag, table.shape[0])
    return emb.double().cpu().numpy()


def _x_device(X, dev):
    """X on the device: f32 rows when X is f32-representable, else f64 rows."""
    X = np.asarray(X)
    if X.ndim != 2:
        raise ValueError(f"Expected 2D array, got {X.ndim}D array instead")
    if X.dtype.kind == "f" and not np.isfinite(X).all():
        raise ValueError("Input X contains NaN." if np.isnan(X).any() else
                         f"Input X contains infinity or a value too large for {X.dtype!r}.")
    x32 = X.astype(np.float32)
    if X.dtype == np.float32 or np.array_equal(x32.astype(X.dtype), X):
        return torch.as_tensor(np.ascontiguousarray(x32)).to(dev)
    return torch.as_tensor(np.ascontiguousarray(X.astype(np.float64))).to(dev)


def _pc_device(x, npc):
    if x.dtype == torch.float64:
        return P.pc_f64(x, npc)
    G = P.gram(x, None)
    z0, transposed = P.pc_start_block(x.shape[0], x.shape[1], npc, x.device, x, None)
    return P.pc_solve(G, z0, npc, transposed)


def compute_pc(X, npc=1):
    """Top-npc right singular vectors, uncentred (DO NOT make X zero-mean)."""
    x = _x_device(X, _dev())
    return _pc_device(x, npc).cpu().numpy()


def remove_pc(X, npc=1):
    """XX = X - X pc^T pc, float64."""
    x = _x_device(X, _dev())
    pc = _pc_device(x, npc)
    if x.dtype == torch.float64:
        return P.remove_pc_f64(x, pc).cpu().numpy()
    return P.remove_pc(x, None, pc, torch.float64).cpu().numpy()


def SIF_embedding(We, x, w, params):
    """Weighted average, then (params.rmpc > 0) first-PC removal — float64 [N, D]."""
    dev = _dev()
    table = _table(We, dev)
    ids = _ids(x, dev)
    wt = torch.as_tensor(np.ascontiguousarray(np.asarray(w, dtype=np.float32))).to(dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    if params.rmpc > 0:
        out, _ = P.sif_embeddings(table, ids, w=wt, npc=params.rmpc, out_dtype=torch.float64,
                                  check_ids=True)
        return out.cpu().numpy()
    emb = P.weighted_sum(table, ids, w=wt, flag=flag, x_out=True)
    P.check_flag(flag, table.shape[0])
    return emb.double().cpu().numpy()
