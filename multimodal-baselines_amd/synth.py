"""Seeded synthetic inputs of the reference's shapes.

The reference ships no GloVe table, no h5 features and no MOSI weights
(`/root/reference/.MISSING_LARGE_BLOBS:1-3`), so every workload here is
synthetic and fully determined by a seed:

* word table   ``E[v] = noise*z_v + common*g`` (one shared direction ``g`` so
  the SIF sentence averages have a dominant first PC, as GloVe averages do —
  the reason SIF removes it, `sif_functions.py:58-81`); row 0 (pad/OOV) = 0.
* token ids    Zipf(s) over ``[1, V)``; optional ragged lengths padded with id 0
  (the reference pads with 0, `simplesif.py:36-40`).
* word weights ``a / (a + p(w))`` with ``a = 1e-3`` (`sif.py:14-32`), ``p`` the
  same Zipf law; ``weights[0]`` configurable (POM ships 1.0, `pom_word_weights.npy`).
* audio/visual dense ``[N, T, F]`` streams, U(-1, 1), optional -10 pads
  (`utils.py:188-189`).

Two back ends with the same recipe: numpy (host fixtures, CPU tests) and torch
on a device (bench: generated in HBM so no H2D sits in the timed region).
"""
from __future__ import annotations

import numpy as np

SIF_A = 1e-3  # sif.py:14 default `a`


def zipf_probs(V: int, s: float = 1.1) -> np.ndarray:
    """p(w) for w in [1, V) normalised; index 0 gets probability 0."""
    r = np.arange(1, V, dtype=np.float64)
    p = r ** (-s)
    p /= p.sum()
    return np.concatenate([[0.0], p])


def sif_weights(V: int, s: float = 1.1, w0: float = 1.0, a: float = SIF_A) -> np.ndarray:
    """SIF weight table a/(a+p(w)) (sif.py:30) as float64, like pom_word_weights.npy."""
    p = zipf_probs(V, s)
    w = a / (a + p)
    w[0] = w0
    return w


def word_table(V: int, D: int = 300, seed: int = 0, noise: float = 0.4,
               common: float = 0.3) -> np.ndarray:
    rng = np.random.default_rng(seed)
    g = rng.standard_normal(D)
    E = noise * rng.standard_normal((V, D)) + common * g
    E = E.astype(np.float32)
    E[0] = 0.0
    return E


def token_ids(N: int, L: int, V: int, seed: int = 0, s: float = 1.1,
              ragged: bool = False, min_len: int = 1) -> np.ndarray:
    """int64 ids [N, L] (the reference id dtype, pom_*_ids.npy)."""
    rng = np.random.default_rng(seed)
    cdf = np.cumsum(zipf_probs(V, s)[1:])
    u = rng.random((N, L))
    ids = np.searchsorted(cdf, u * cdf[-1], side="right") + 1
    ids = np.minimum(ids, V - 1).astype(np.int64)
    if ragged:
        lens = rng.integers(min_len, L + 1, size=N)
        ids[np.arange(L)[None, :] >= lens[:, None]] = 0
    return ids


def frames(N: int, T: int, F: int, seed: int = 0, pad_frac: float = 0.0) -> np.ndarray:
    """float32 [N, T, F] U(-1,1); trailing pad frames set to -10 (utils.py:188-189)."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(-1.0, 1.0, size=(N, T, F)).astype(np.float32)
    if pad_frac > 0:
        npad = rng.integers(0, max(1, int(T * pad_frac)) + 1, size=N)
        for i in range(N):
            if npad[i]:
                x[i, T - npad[i]:, :] = -10.0
    return x


# ---------------------------------------------------------------- device side
def device_workload(N: int, T: int, V: int, D: int = 300, A: int = 300, Vd: int = 300,
                    seed: int = 0, device="cuda", s: float = 1.1, w0: float = 1.0,
                    mean_len: float | None = None, poisson_len: float | None = None):
    """Config-3 workload generated directly in device memory (torch RNG).

    Returns dict of device tensors: table [V,D] f32, wtab [V] f32 (the f32
    rounding of the f64 SIF weights, as `simplesif.py:315` does), ids [N,T]
    int32, audio [N,T,A] f32, visual [N,T,Vd] f32.

    Ragged variants (pad tokens id 0, pad frames -10, utils.py:188-189):
    `mean_len` -- POM-like lengths ~ N(mean, mean/1.5) clipped to [1, T];
    `poisson_len` -- SURVEY §8d's second configs[3] run, Poisson(mean) lengths
    clipped to [1, T] (T = 64 there).  The result then also holds `lengths` [N].
    """
    import torch

    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    g = torch.randn(D, generator=gen, device=device, dtype=torch.float32)
    table = torch.randn(V, D, generator=gen, device=device, dtype=torch.float32)
    table.mul_(0.4).add_(0.3 * g)
    table[0].zero_()
    p = torch.tensor(zipf_probs(V, s), device=device, dtype=torch.float64)
    wtab = (SIF_A / (SIF_A + p)).to(torch.float32)
    wtab[0] = w0
    cdf = torch.cumsum(p[1:], 0)
    ids = torch.empty(N, T, device=device, dtype=torch.int32)
    chunk = 1 << 22
    flat = ids.view(-1)
    for o in range(0, flat.numel(), chunk):
        n = min(chunk, flat.numel() - o)
        u = torch.rand(n, generator=gen, device=device, dtype=torch.float64) * cdf[-1]
        flat[o:o + n] = (torch.searchsorted(cdf, u, right=True) + 1).clamp_(max=V - 1).to(torch.int32)
    audio = torch.empty(N, T, A, device=device, dtype=torch.float32)
    visual = torch.empty(N, T, Vd, device=device, dtype=torch.float32)
    audio.uniform_(-1.0, 1.0, generator=gen)
    visual.uniform_(-1.0, 1.0, generator=gen)
    out = {"table": table, "wtab": wtab, "ids": ids, "audio": audio, "visual": visual}
    lens = None
    if mean_len is not None:
        # ragged transcripts padded to T (POM: 370 / 325 mean non-pad ids of 1089 /
        # 1357): lengths ~ N(mean, mean/1.5) clipped to [1, T]; pad
        # tokens are id 0 (weight w0, counted like the reference) and pad frames -10
        lens = (torch.randn(N, generator=gen, device=device) * (mean_len / 1.5) + mean_len)
        lens = lens.round().clamp_(1, T).to(torch.int64)
    elif poisson_len is not None:
        rate = torch.full((N,), float(poisson_len), device=device)
        lens = torch.poisson(rate, generator=gen).clamp_(1, T).to(torch.int64)
    if lens is not None:
        for o in range(0, N, 1 << 16):  # bounded temporaries
            sl = slice(o, min(N, o + (1 << 16)))
            pad = torch.arange(T, device=device)[None, :] >= lens[sl, None]
            ids[sl].masked_fill_(pad, 0)
            audio[sl].masked_fill_(pad[:, :, None], -10.0)
            visual[sl].masked_fill_(pad[:, :, None], -10.0)
        out["lengths"] = lens
    return out


SHARD_BLOCK = 62_500  # rows per seeded block of a sharded workload (1M / 16)


def device_shard(row0: int, n: int, T: int, V: int, D: int = 300, A: int = 300, Vd: int = 300,
                 seed: int = 1000, device="cuda", block: int = SHARD_BLOCK):
    """Rows [row0, row0 + n) of ONE synthetic config-3 split, generated in
    device memory the same way whatever the sharding: the word table and
    weights come from `seed` (replicated on every rank), the utterances from
    seeded blocks of `block` rows (block b: seed + 1 + b).  So the N shards of
    bench.py's strong scaling (1M / N rows each) are slices of the same
    1M-utterance split for every N, and a test can rebuild the union of the
    ranks' rows in one process.  Same recipe as device_workload (Zipf ids,
    U(-1, 1) frames); returns the same dict."""
    import torch

    base = device_workload(1, T, V, D=D, A=1, Vd=1, seed=seed, device=device)
    ids = torch.empty(n, T, device=device, dtype=torch.int32)
    audio = torch.empty(n, T, A, device=device, dtype=torch.float32)
    visual = torch.empty(n, T, Vd, device=device, dtype=torch.float32)
    r = row0
    while r < row0 + n:
        b = r // block
        b0 = b * block
        hi = min(row0 + n, b0 + block)
        # the whole block from its seed (device RNG streams are not
        # prefix-stable across sizes), then the rows this shard owns
        blk = device_workload(block, T, V, D=1, A=A, Vd=Vd, seed=seed + 1 + b, device=device)
        ids[r - row0:hi - row0] = blk["ids"][r - b0:hi - b0]
        audio[r - row0:hi - row0] = blk["audio"][r - b0:hi - b0]
        visual[r - row0:hi - row0] = blk["visual"][r - b0:hi - b0]
        del blk
        r = hi
    return {"table": base["table"], "wtab": base["wtab"], "ids": ids, "audio": audio,
            "visual": visual}


# ---------------------------------------------------------------- CLI datasets
def mm_splits(seed: int = 0, sizes=(96, 32, 32), T: int = 12, V: int = 300, A_raw: int = 20,
              Vd_raw: int = 14, dataset: str = "mosi", n_labels: int = 1):
    """Seeded splits in the layout `utils.load_data` returns (utils.py:20-90):
    (word2ix, word_embeddings [V, 300] f32, (train, valid, test)), each split a
    dict of numpy arrays.

    mosi: facet [N,T,Vd_raw], covarep [N,T,A_raw], text [N,T] aligned ids
          (left-padded with 0), lengths, label [N], id.
    pom:  facet, covarep, text [N,T,300] aligned text embeddings (0 rows at
          pads), label [N, n_labels], text_id [N, L_text] unaligned ids.
    Raw frames are 0 at padded time steps (what normalize_data turns into the
    -10 pads, utils.py:171-189); covarep feature 1 is constant 0 in every split
    (dropped by normalize_data, utils.py:163-169).
    """
    rng = np.random.default_rng(seed)
    E = word_table(V, 300, seed=seed + 1)
    word2ix = {f"w{i}": i for i in range(V)}
    splits = []
    for N in sizes:
        lens = rng.integers(max(1, T // 3), T + 1, size=N)
        pad = np.arange(T)[None, :] < (T - lens)[:, None]          # left padding
        ids = rng.integers(1, V, size=(N, T)).astype(np.int64)
        ids[pad] = 0
        cov = rng.normal(0.0, 1.0, size=(N, T, A_raw)).astype(np.float32)
        fac = rng.normal(0.5, 1.0, size=(N, T, Vd_raw)).astype(np.float32)
        cov[pad] = 0.0
        fac[pad] = 0.0
        cov[:, :, 1] = 0.0
        if n_labels == 1 and dataset == "mosi":
            label = rng.uniform(-3.0, 3.0, size=N).astype(np.float32)
        else:
            label = rng.uniform(1.0, 7.0, size=(N, n_labels)).astype(np.float32)
        d = {"facet": fac, "covarep": cov, "label": label}
        if dataset == "mosi":
            d.update(text=ids, lengths=lens.astype(np.int64), id=np.arange(N).astype(np.int64))
        else:
            d["text"] = np.where(pad[:, :, None], 0.0, E[ids]).astype(np.float32)
            Lt = T + 3
            tid = rng.integers(1, V, size=(N, Lt)).astype(np.int64)
            tl = rng.integers(2, Lt + 1, size=N)
            tid[np.arange(Lt)[None, :] >= tl[:, None]] = 0
            d["text_id"] = tid
        splits.append(d)
    return word2ix, E, tuple(splits)


# ---------------------------------------------------------------- per-split (real call pattern)
MOSI_SPLITS = (1284, 229, 686)  # train / valid / test utterances (SURVEY.md §8 shapes)


def split_arrays(ids: np.ndarray, E: np.ndarray, wt: np.ndarray, A: int, Vd: int,
                 seed: int) -> dict:
    """Host arrays of one split: ids [N, L] int64, the word table, the f64
    weights, and aligned audio / visual frames [N, L, A|Vd] (U(-1, 1), -10 at
    the time steps past each utterance's last non-zero id, utils.py:188-189)."""
    n, L = ids.shape
    rng = np.random.default_rng(seed)
    nz = ids != 0
    lens = np.where(nz.any(1), L - np.argmax(nz[:, ::-1], axis=1), 0)
    pad = np.arange(L)[None, :] >= lens[:, None]
    out = {"ids": ids, "table": E, "weights": wt}
    for key, F in (("audio", A), ("visual", Vd)):
        x = rng.uniform(-1.0, 1.0, size=(n, L, F)).astype(np.float32)
        x[pad] = -10.0
        out[key] = x
    return out


def mosi_splits(sizes=MOSI_SPLITS, L: int = 20, V: int = 3016, A: int = 76, Vd: int = 48,
                seed: int = 21) -> list[dict]:
    """configs[0]/[1] at their real call pattern: three MOSI-shaped splits
    (1284 / 229 / 686 utterances, L = T = 20, V = 3016, COVAREP 74 + 2 and
    FACET 46 + 2 positional dims) sharing one word table and weight table
    (w0 = 0: MOSI pads carry no weight); ragged transcripts."""
    E = word_table(V, 300, seed=seed)
    wt = sif_weights(V, w0=0.0)
    return [split_arrays(token_ids(n, L, V, seed=seed + 1 + i, ragged=True), E, wt, A, Vd,
                         seed=seed + 11 + i) for i, n in enumerate(sizes)]


def pom_splits(valid_ids, test_ids, weights, table_seed: int, A: int = 300,
               Vd: int = 300) -> list[dict]:
    """configs[2] at its real call pattern: the reference's own POM valid /
    test id matrices (100 x 1089, 203 x 1357) and weights, the seeded V = 7763
    word table (GloVe is absent), aligned frames of the transcripts' length."""
    E = word_table(len(weights), 300, seed=table_seed)
    return [split_arrays(np.asarray(ids, np.int64), E, np.asarray(weights, np.float64), A, Vd,
                         seed=table_seed + 1 + i) for i, ids in enumerate((valid_ids, test_ids))]


def to_device(split: dict, device) -> dict:
    """A split's FusedStep inputs on the device (ids int32, wtab = the f32
    rounding of the f64 weights, simplesif.py:315)."""
    import torch

    return {"table": torch.as_tensor(split["table"]).to(device),
            "wtab": torch.as_tensor(split["weights"], dtype=torch.float32).to(device),
            "ids": torch.as_tensor(split["ids"], dtype=torch.int32).to(device),
            "audio": torch.as_tensor(split["audio"]).to(device),
            "visual": torch.as_tensor(split["visual"]).to(device)}
