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
    """sif.py:14-32 — weight(word) = a / (a + count/N) from a 'word count' file."""
    word_weights = {}
    N = 0
    with open(word_freq_file, "r") as f:
        for line in f:
            line = line.strip()
            if len(line) > 0:
                line = line.split()
                if len(line) == 2:
                    word_weights[line[0]] = float(line[1])
                    N += float(line[1])
                else:
                    print(line)
    for key, value in word_weights.items():
        word_weights[key] = a / (a + value / N)
    return word_weights


def load_weights(args):
    """sif.py:34-42."""
    if args["dataset"] == "mosi":
        return load_mosi_weights()
    elif args["dataset"] == "pom":
        return load_pom_weights()
    elif args["dataset"] == "iemocap":
        return load_iemocap_weights()
    raise NotImplementedError


def load_pom_weights():
    weights = np.load("pom/pom_word_weights.npy").squeeze()
    print(weights.shape)
    return weights


def load_iemocap_weights():
    weights = np.load("iemocap/iemocap_word_weights.npy").squeeze()
    print(weights.shape)
    return weights


def load_mosi_weights(word2ix=None, word_freq_file="SIF/auxiliary_data/enwiki_vocab_min200.txt"):
    """sif.py:52-76.  The reference regenerates word_weights.npy from a word
    frequency file using a `word2ix` it never defines (sif.py:63, NameError);
    here the mapping is an explicit argument and the same rule is applied
    (unknown words weigh 1.0)."""
    if os.path.isfile("word_weights.npy"):
        return np.load("word_weights.npy", allow_pickle=False).squeeze()
    if word2ix is None:
        raise NameError("word_weights.npy is absent and no word2ix mapping was given "
                        "(the reference fails here too: sif.py:63)")
    word_weights = get_word_weights(word_freq_file)
    weights = np.zeros((max(word2ix.values()) + 1))
    unk = 0
    for word, ix in word2ix.items():
        if word.lower() not in word_weights:
            weights[ix] = 1.0
            unk += 1
        else:
            weights[ix] = word_weights[word.lower()]
    print("# of words with unknown weight", unk)
    np.save("word_weights.npy", weights, allow_pickle=False)
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
