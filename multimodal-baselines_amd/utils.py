"""Drop-in for `/root/reference/utils.py` — data loading and preprocessing.

Host-side numpy, as in the reference (one pass per split, before any device
work), with the reference's behaviour kept quirk for quirk (SURVEY.md §8
"Parity traps"):

* `normalize_data` drops covarep features that are constant over the split,
  then maps x -> (x + min) * 2 / (max - min) - 1 (the reference's "+ min",
  utils.py:185-186), leaves a zero range unguarded for facet, and sets the
  padding entries (raw value 0) to -10; masks are taken before normalising.
* `add_positional_embeddings` writes sin/cos into the UTTERANCE axis rows
  2i / 2i+1 of the index block (utils.py:146-148), so only utterances
  0 .. pos_embed_dim-1 get sin/cos and every other utterance carries the raw
  frame index in all pos_embed_dim columns.

Data files are read with the same names and layout as the reference
(`data/{mosi,pom}_data.h5`, `data/iemocap_<emotion>.h5` via h5py, the .npy id
and table files via numpy with allow_pickle=False, `word2ix` pickles / json).
h5py is optional: when it is not installed, an `.npz` holding the same arrays
under `<split>/<key>` names (`data/mosi_data.npz`, ...) is read instead.
"""
from __future__ import annotations

import json
import os
import pickle

import numpy as np
import torch
from torch.utils.data import Dataset

H5_KEYS = {
    "mosi": ("facet", "covarep", "text", "lengths", "label", "id"),
    "pom": ("facet", "covarep", "text", "label"),
    "iemocap": ("facet", "covarep", "text", "label"),
}


def _read_splits(path_h5: str, keys) -> tuple[dict, dict, dict]:
    """train/valid/test dicts of `keys` from an h5 file (utils.py:35-48) or
    from the .npz twin `<split>/<key>` when h5py is absent."""
    out = ({}, {}, {})
    names = ("train", "valid", "test")
    try:
        import h5py  # noqa: F401
        have_h5 = hasattr(h5py, "File")
    except ImportError:
        have_h5 = False
    if have_h5 and os.path.exists(path_h5):
        import h5py

        with h5py.File(path_h5, "r") as f:
            for k in keys:
                for d, s in zip(out, names):
                    d[k] = f[s][k][:]
        return out
    npz = os.path.splitext(path_h5)[0] + ".npz"
    if os.path.exists(npz):
        with np.load(npz, allow_pickle=False) as z:
            for k in keys:
                for d, s in zip(out, names):
                    d[k] = z[f"{s}/{k}"]
        return out
    if not have_h5 and os.path.exists(path_h5):
        raise ImportError(f"{path_h5} needs h5py, which is not installed (or provide {npz})")
    raise FileNotFoundError(path_h5)


def save_splits_npz(path: str, splits) -> None:
    """Write train/valid/test dicts as the `.npz` twin _read_splits accepts."""
    arrs = {}
    for d, s in zip(splits, ("train", "valid", "test")):
        for k, v in d.items():
            arrs[f"{s}/{k}"] = np.asarray(v)
    np.savez(path, **arrs)


def load_data(args):
    """utils.py:10-18."""
    if args["dataset"] == "mosi":
        return load_mosi()
    elif args["dataset"] == "pom":
        return load_pom()
    elif args["dataset"] == "iemocap":
        return load_iemocap(args)
    raise ValueError


def load_mosi():
    """utils.py:20-50."""
    with open("mosi/word2ix_300_mosi.pkl", "rb") as f:
        word2ix = pickle.load(f)  # the dataset's own file, as in the reference
    word_embeddings = np.load("mosi/glove_300_mosi.npy", allow_pickle=False)
    train, valid, test = _read_splits("data/mosi_data.h5", H5_KEYS["mosi"])
    return word2ix, word_embeddings, (train, valid, test)


def _with_text_ids(prefix, splits):
    for d, s in zip(splits, ("train", "valid", "test")):
        d["text_id"] = np.load(f"{prefix}_{s}_ids.npy", allow_pickle=False)
    return splits


def load_pom():
    """utils.py:52-90 (ids of the unaligned transcript from pom/pom_*_ids.npy)."""
    with open("pom/glove_mappings.pom.json") as f:
        word2ix = json.load(f)
    word_embeddings = np.load("pom/glove.pom.npy", allow_pickle=False)
    splits = _read_splits("data/pom_data.h5", H5_KEYS["pom"])
    print(splits[0]["text"].shape)
    return word2ix, word_embeddings, _with_text_ids("pom/pom", splits)


def load_iemocap(args):
    """utils.py:92-128."""
    with open("iemocap/glove_mappings.iemocap.json") as f:
        word2ix = json.load(f)
    word_embeddings = np.load("iemocap/glove.iemocap.npy", allow_pickle=False)
    splits = _read_splits("data/iemocap_{}.h5".format(args["emotion"]), H5_KEYS["iemocap"])
    print(splits[0]["text"].shape)
    return word2ix, word_embeddings, _with_text_ids("iemocap/iemocap", splits)


def add_positional_embeddings(args, data):
    """utils.py:130-153: appends pos_embed_dim columns to data [N, T, F].

    The block starts as the frame index t in every column; then for
    i < pos_embed_dim // 2 the reference overwrites block[2i] and block[2i+1]
    — indexing the first (utterance) axis — with sin / cos of
    t / 10000^(2i / pos_embed_dim).
    """
    n, t = data.shape[0], data.shape[1]
    pe = args["pos_embed_dim"]
    block = np.broadcast_to(np.arange(t, dtype=np.float32)[None, :, None], (n, t, pe)).copy()
    for i in range(pe // 2):
        div = 10000 ** (2 * i / pe)
        if 2 * i < n:
            block[2 * i] = np.sin(block[2 * i] / div)
        if 2 * i + 1 < n:
            block[2 * i + 1] = np.cos(block[2 * i + 1] / div)
    return np.concatenate([data, block], axis=-1)


def normalize_data(train):
    """utils.py:155-191: in-place on the split dict; returns (split, masks)."""
    cov = train["covarep"]
    keep = (cov.max((0, 1)) - cov.min((0, 1))).nonzero()[0]
    cov = cov[:, :, keep]
    fac = train["facet"]
    cov_pad, fac_pad = cov == 0, fac == 0
    masks = {"covarep": (~cov_pad).astype(int), "facet": (~fac_pad).astype(int)}
    a_lo, a_hi = cov.min((0, 1)), cov.max((0, 1))
    v_lo, v_hi = fac.min((0, 1)), fac.max((0, 1))
    cov = (cov + a_lo) * 2. / (a_hi - a_lo) - 1.
    fac = (fac + v_lo) * 2. / (v_hi - v_lo) - 1.
    cov[cov_pad] = -10.
    fac[fac_pad] = -10.
    train["covarep"], train["facet"] = cov, fac
    return train, masks


class MMData(Dataset):
    """utils.py:193-233: per-split device tensors; items are
    (idx, text, audio, visual, text_mask, audio_mask, visual_mask, text_weights)."""

    def __init__(self, text, audio, visual, masks, text_weights, device):
        super(Dataset, self).__init__()
        t = lambda x: x if torch.is_tensor(x) else torch.tensor(x, device=device, dtype=torch.float32)
        text, text_weights, audio, visual = t(text), t(text_weights), t(audio), t(visual)
        tm = {k: t(masks[k]) for k in ("text", "covarep", "facet")}
        assert text.size()[0] == audio.size()[0]
        assert audio.size()[0] == visual.size()[0]
        assert text.size()[0] == text_weights.size()[0]
        self.text, self.text_weights, self.audio, self.visual = text, text_weights, audio, visual
        self.text_mask, self.audio_mask, self.visual_mask = tm["text"], tm["covarep"], tm["facet"]
        self.len = self.text.size()[0]

    def __len__(self):
        return self.len

    def __getitem__(self, idx):
        return (idx, self.text[idx], self.audio[idx], self.visual[idx], self.text_mask[idx],
                self.audio_mask[idx], self.visual_mask[idx], self.text_weights[idx])


class MMDataExtra(MMData):
    """utils.py:235-251: adds the aligned text and its mask (POM / IEMOCAP)."""

    def __init__(self, text, audio, visual, masks, text_weights, text_aligned, device):
        super().__init__(text, audio, visual, masks, text_weights, device)
        if not torch.is_tensor(text_aligned):
            text_aligned = torch.tensor(text_aligned, device=device, dtype=torch.float32)
        self.text_aligned = text_aligned
        self.text_aligned_mask = torch.tensor(masks["text_align"], device=device, dtype=torch.float32)

    def __getitem__(self, idx):
        return super().__getitem__(idx) + (self.text_aligned[idx], self.text_aligned_mask[idx])
