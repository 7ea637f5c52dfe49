"""CPU restatement of the SIF text-embedding path (a1-a5) — TEST INFRASTRUCTURE ONLY.

Follows `/root/reference/sif_functions.py` and `/root/reference/sif.py`.  The PC
step restates scikit-learn's `TruncatedSVD(algorithm='randomized')`
(third-party; the reference pins no version — this image has scikit-learn
1.7.2: `sklearn/decomposition/_truncated_svd.py:fit_transform`,
`sklearn/utils/extmath.py:_randomized_range_finder` / `_randomized_svd`).
"""
from __future__ import annotations

import numpy as np
from scipy import linalg


def seq2weight(seq, mask, weight4ind):
    """sif_functions.py:8-15 — per-token weight gather, f64 table -> f32 output.

    Vectorised form of the reference double loop: weight = table[id] where
    mask > 0 and id >= 0, else 0.
    """
    seq = np.asarray(seq)
    sel = (np.asarray(mask) > 0) & (seq >= 0)
    out = np.zeros(seq.shape, dtype=np.float32)
    out[sel] = np.asarray(weight4ind)[seq[sel]]
    return out


def seq2weight_loop(seq, mask, weight4ind):
    """The literal loop of sif_functions.py:10-13 (small inputs only)."""
    w = np.zeros(seq.shape).astype("float32")
    for i in range(seq.shape[0]):
        for j in range(seq.shape[1]):
            if mask[i, j] > 0 and seq[i, j] >= 0:
                w[i, j] = weight4ind[seq[i, j]]
    return w


def get_weighted_average(We, x, w):
    """sif_functions.py:28-56 — emb[i] = w[i].dot(We[x[i]]) / count_nonzero(w[i]).

    Output float64 (np.zeros default, :37); each row is computed in the table's
    dtype (f32 sgemv for an f32 table) exactly as the reference row loop does.
    Negative ids wrap (numpy fancy indexing) — with weight 0 they add nothing.
    """
    n = x.shape[0]
    emb = np.zeros((n, We.shape[1]))
    for i in range(n):
        emb[i, :] = w[i, :].dot(We[x[i, :], :]) / np.count_nonzero(w[i, :])
    return emb


# --------------------------------------------------------------------- PC (a3)
def randomized_svd_components(M, n_components, n_oversamples=10, n_iter=7, random_state=0):
    """Restates sklearn 1.7.2 `_randomized_svd` + TruncatedSVD's svd_flip.

    * transpose when n_samples < n_features (extmath.py:562-566);
    * Q ~ RandomState(seed).normal(size=(M.shape[1], k+p)), cast to M's float
      dtype (extmath.py:297-301);
    * n_iter rounds of LU(permute_l) normalised power iteration
      (normalizer 'auto' -> 'LU' for n_iter > 2, extmath.py:313-352);
    * QR, B = Q^T M, SVD of B (gesdd), U = Q Uhat (extmath.py:354-590);
    * TruncatedSVD passes flip_sign=False then svd_flip(U, VT,
      u_based_decision=False) (_truncated_svd.py:244-253).
    Returns components_ [n_components, n_features].
    """
    rs = np.random.RandomState(random_state)
    A = M
    n_samples, n_features = A.shape
    k = n_components + n_oversamples
    transpose = n_samples < n_features
    if transpose:
        A = A.T
    Q = rs.normal(size=(A.shape[1], k))
    if A.dtype.kind == "f":
        Q = Q.astype(A.dtype, copy=False)
    for _ in range(n_iter):
        Q, _ = linalg.lu(A @ Q, permute_l=True, check_finite=False)
        Q, _ = linalg.lu(A.T @ Q, permute_l=True, check_finite=False)
    Q, _ = linalg.qr(A @ Q, mode="economic", check_finite=False)
    B = Q.T @ A
    Uhat, s, Vt = linalg.svd(B, full_matrices=False, lapack_driver="gesdd")
    U = Q @ Uhat
    if transpose:
        U, Vt = Vt[:n_components, :].T, U[:, :n_components].T
    else:
        U, Vt = U[:, :n_components], Vt[:n_components, :]
    # svd_flip(u, v, u_based_decision=False): largest |v| entry of each row > 0
    idx = np.argmax(np.abs(Vt), axis=1)
    signs = np.sign(Vt[np.arange(Vt.shape[0]), idx])
    return Vt * signs[:, None]


def compute_pc(X, npc=1):
    """sif_functions.py:58-67 (uncentred; TruncatedSVD(npc, n_iter=7, random_state=0))."""
    return randomized_svd_components(np.asarray(X), npc, n_oversamples=10, n_iter=7,
                                     random_state=0)


def remove_pc(X, npc=1):
    """sif_functions.py:69-81."""
    pc = compute_pc(X, npc)
    if npc == 1:
        return X - X.dot(pc.transpose()) * pc
    return X - X.dot(pc.transpose()).dot(pc)


def SIF_embedding(We, x, w, rmpc=1):
    """sif_functions.py:84-96."""
    emb = get_weighted_average(We, x, w)
    if rmpc > 0:
        emb = remove_pc(emb, rmpc)
    return emb


def get_sentence_embeddings(word_embeddings, weights, text):
    """sif.py:78-94 — mask = ones, rmpc = 1."""
    w = seq2weight(text, np.ones(text.shape), weights)
    return SIF_embedding(word_embeddings, text, w, 1)


def _orth(Z):
    """Modified Gram-Schmidt, twice (the device solver's orthonormalisation)."""
    Z = np.array(Z, dtype=np.float64, copy=True)
    for j in range(Z.shape[1]):
        for _ in range(2):
            for i in range(j):
                Z[:, j] -= (Z[:, i] @ Z[:, j]) * Z[:, i]
        Z[:, j] /= np.linalg.norm(Z[:, j])
    return Z


def pc_from_gram(G, z0, npc=1, transposed=False, n_iter=7):
    """CPU restatement of the DEVICE solver (csrc/pc_kernels.hip, mmb_pc_solve):
    sklearn's randomized SVD evaluated from the Gram G = X^T X alone.

    The reference's iterations build span(G^n_iter Omega) (direct branch) or
    span(G^n_iter X^T Omega) (transposed branch, n < d): LU / QR normalisers
    only right-multiply the block, so the span is exact algebra.  Direct: the
    top right singular vectors of Q^T X, Q = orth(X Z), solve
    (Z^T G^2 Z) y = s^2 (Z^T G Z) y, v = G Z y.  Transposed: v = Z u, u the
    top eigenvectors of Z^T G Z.  svd_flip(u_based_decision=False) at the end.
    """
    G = np.asarray(G, np.float64)
    Z = _orth(z0)
    for _ in range(n_iter):
        Z = _orth(G @ Z)
    GZ = G @ Z
    if transposed:
        lam, U = np.linalg.eigh(Z.T @ GZ)
        V = Z @ U[:, ::-1][:, :npc]
    else:
        W = Z.T @ GZ
        H = GZ.T @ GZ
        Li = np.linalg.inv(np.linalg.cholesky(0.5 * (W + W.T)))
        lam, U = np.linalg.eigh(Li @ (0.5 * (H + H.T)) @ Li.T)
        V = GZ @ (Li.T @ U[:, ::-1][:, :npc])
    V = (V / np.linalg.norm(V, axis=0)).T
    idx = np.argmax(np.abs(V), axis=1)
    return V * np.sign(V[np.arange(V.shape[0]), idx])[:, None]


def sliced_gram(X, colmax=None):
    """CPU restatement of the int8 Gram (csrc/pc_kernels.hip gram_i8l_kernel;
    r04's gram_i8_kernel had the same digits and pairs): each value a 30-bit
    fixed-point integer of its column's power-of-two bound 2^e (|x| <= colmax
    < 2^e), v = rint(x 2^(30-e)), cut into four balanced base-256 digits (top
    in [-64, 64]); digit-pair products of level a + b <= 4 summed exactly,
    G = 2^(e_i + e_j - 60) sum over those pairs.  (The device sums each level
    exactly in int32 over a row range and rounds each range's combination
    once; here every pair's exact integer sum is rounded once: the two agree
    to the f64 summation of the range partials, ~1e-16.)  Test
    infrastructure: the reference has no counterpart (its TruncatedSVD works
    on X itself); this pins the device kernel's arithmetic."""
    X = np.asarray(X, np.float32).astype(np.float64)
    m = np.abs(X).max(0) if colmax is None else np.asarray(colmax, np.float64)
    e = np.where(m > 0, np.frexp(m)[1], 0).astype(np.int64)
    v = np.rint(np.ldexp(X, 30 - e[None, :])).astype(np.int64)
    digs = []
    for _ in range(4):
        lo = ((v + 128) & 255) - 128
        digs.append(lo)
        v = (v - lo) >> 8
    assert (v == 0).all()
    digs = [d.astype(np.float64) for d in digs[::-1]]  # top digit first
    assert np.abs(digs[0]).max(initial=0) <= 64
    G = np.zeros((X.shape[1],) * 2)
    for a in range(4):
        for b in range(4):
            if a + b <= 4:
                G += (digs[a].T @ digs[b]) * 2.0 ** (8 * (6 - a - b) - 60)
    return G * np.ldexp(1.0, e[:, None] + e[None, :])


class CPUOps:
    """CPU doubles of the libmmb kernels that pipeline.global_pc composes
    (torch CPU tensors in/out) — lets the multi-rank orchestration run under
    gloo in tests."""

    @staticmethod
    def gram(num, cnt, G=None, ws=None):
        import torch

        x = (num / cnt[:, None]) if cnt is not None else num
        x = x.to(torch.float64)
        return x.T @ x

    @staticmethod
    def omega(rows, k, device=None):
        import torch

        return torch.from_numpy(np.random.RandomState(0).normal(size=(rows, k)))

    @staticmethod
    def xt_omega(num, cnt, om):
        x = (num / cnt[:, None]) if cnt is not None else num
        return x.double().T @ om

    @staticmethod
    def pc_solve(G, z0, npc, transposed):
        import torch

        return torch.from_numpy(pc_from_gram(G.numpy(), z0.numpy(), npc, transposed))


def exact_top_pc(X, npc=1):
    """Exact top right singular vectors (for the spectral-gap discussion only)."""
    _, _, vt = np.linalg.svd(np.asarray(X, np.float64), full_matrices=False)
    v = vt[:npc]
    idx = np.argmax(np.abs(v), axis=1)
    return v * np.sign(v[np.arange(npc), idx])[:, None]
