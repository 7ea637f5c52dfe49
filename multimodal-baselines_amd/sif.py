"""Drop-in for `/root/reference/sif.py` — SIF word weights and per-split sentence embeddings.

Host-side file handling (word-frequency file, .npy weight tables) keeps the
reference's behaviour; the per-utterance arithmetic runs on the GPU:
`get_sentence_embeddings` is a1-a5 fused on device (weights gathered by id
inside the gather-reduce kernel, never materialised).
"""
from __future__ import annotations

import os

import numpy as np
import torch

import mmb_lib as L
import pipeline as P
from sif_functions import seq2weight


def get_word_weights(word_freq_file, a=1e-3):
    """sif.py:14-32 -- SIF weight a / (a + p(w)) with p(w) = count / total count,
    read from a "word count" file.  Blank lines are skipped; a line that is not
    exactly two fields is echoed (as the list of its fields) and ignored; a word
    listed twice keeps its last count but both counts enter the total."""
    counts = {}
    total = 0.0
    with open(word_freq_file, "r") as fh:
        for fields in (ln.split() for ln in fh):
            if not fields:
                continue
            if len(fields) != 2:
                print(fields)
                continue
            word, c = fields[0], float(fields[1])
            counts[word] = c
            total += c
    return {word: a / (a + c / total) for word, c in counts.items()}


# dataset -> the .npy weight table the reference loads (sif.py:34-50)
_WEIGHT_FILES = {"pom": "pom/pom_word_weights.npy", "iemocap": "iemocap/iemocap_word_weights.npy"}


def _load_table(path):
    table = np.load(path).squeeze()
    print(table.shape)
    return table


def load_weights(args):
    """sif.py:34-42: the dataset's word-weight table (NotImplementedError for
    any other dataset name)."""
    name = args["dataset"]
    if name == "mosi":
        return load_mosi_weights()
    if name in _WEIGHT_FILES:
        return _load_table(_WEIGHT_FILES[name])
    raise NotImplementedError


def load_pom_weights():
    return _load_table(_WEIGHT_FILES["pom"])


def load_iemocap_weights():
    return _load_table(_WEIGHT_FILES["iemocap"])


def load_mosi_weights(word2ix=None, word_freq_file="SIF/auxiliary_data/enwiki_vocab_min200.txt"):
    """sif.py:52-76.  The reference regenerates word_weights.npy from a word
    frequency file using a `word2ix` it never defines (sif.py:63, NameError);
    here the mapping is an explicit argument and the same rule is applied
    (lower-cased lookup; unknown words weigh 1.0)."""
    cached = "word_weights.npy"
    if os.path.isfile(cached):
        return np.load(cached, allow_pickle=False).squeeze()
    if word2ix is None:
        raise NameError("word_weights.npy is absent and no word2ix mapping was given "
                        "(the reference fails here too: sif.py:63)")
    freq = get_word_weights(word_freq_file)
    weights = np.zeros(max(word2ix.values()) + 1)  # indices no word maps to stay 0
    n_unknown = 0
    for word, ix in word2ix.items():  # later entries win on a shared index, as in the reference
        w = freq.get(word.lower())
        n_unknown += w is None
        weights[ix] = 1.0 if w is None else w
    print("# of words with unknown weight", n_unknown)
    np.save(cached, weights, allow_pickle=False)
    return weights


def get_sentence_word_weights(text, weights):
    """sif.py:78-82 — seq2weight with an all-ones mask (bit-exact)."""
    return seq2weight(text, np.ones(np.asarray(text).shape), weights)


def get_sentence_embeddings(word_embeddings, weights, text):
    """sif.py:84-94 — SIF embedding with the first PC removed (rmpc = 1), float64."""
    dev = L.require_gpu()
    table = torch.as_tensor(np.ascontiguousarray(np.asarray(word_embeddings, dtype=np.float32))).to(dev)
    wtab32 = torch.as_tensor(np.asarray(weights, dtype=np.float64).astype(np.float32)).to(dev)
    text = np.asarray(text)
    if text.dtype.kind not in "iu":
        raise IndexError("arrays used as indices must be of integer type")
    ids = P.narrow_ids(torch.from_numpy(np.ascontiguousarray(text, dtype=np.int64)).to(dev))
    out, _ = P.sif_embeddings(table, ids, wtab32=wtab32, npc=1, out_dtype=torch.float64)
    return out.cpu().numpy()
