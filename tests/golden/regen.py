"""Seeded fixture arrays rebuilt from their recipes (r03 fixture slimming).

tests/golden/slim_goldens.py drops an array from a fixture only after the
recipe here rebuilt it bit for bit; it records the array's sha256 as
`<key>__sha256`, and tests/conftest.py's loader rebuilds the array on access
and checks the hash.  The recipes are the generators the make_goldens*.py
scripts fed to the reference (numpy's default_rng streams and torch's CPU
generator are platform independent), plus one recorded-output case:

* emb (g1*, g2, g3, g3b): the reference's a2 rows (sif_functions.py:28-56,
  an f32 sgemv per row, so BLAS-kernel dependent) = the BLAS-free sequential
  f32 accumulation below + a stored int32 ULP residual `emb__resid` (mostly
  zeros: compresses ~8x).
"""
import hashlib
import os
import sys

import numpy as np

_PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                    "multimodal-baselines_amd")
if _PKG not in sys.path:
    sys.path.insert(0, _PKG)


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def table(z):
    import synth

    E = synth.word_table(int(z["V"]), int(z["D"]) if "D" in z else 300, seed=int(z["table_seed"]),
                         common=float(z["common"]) if "common" in z else 0.3)
    assert float(np.asarray(E, np.float64).sum()) == float(z["table_checksum"]), "table checksum"
    return E


def emb_sequential(E, ids, w):
    """Row i: sum_l w[i, l] E[ids[i, l]] accumulated in f32 in token order,
    divided by the nonzero-weight count in f32 -- numpy elementwise only."""
    acc = np.zeros((ids.shape[0], E.shape[1]), np.float32)
    for t in range(ids.shape[1]):
        acc = acc + w[:, t:t + 1] * E[ids[:, t]]
    return acc / np.count_nonzero(w, axis=1)[:, None].astype(np.float32)


def seq_weights(z, ids_key="ids"):
    """The a1 weights: the fixture's own `w`, or (g3b) the reference's
    get_sentence_word_weights restated (weights[id], 0 where id < 0)."""
    if "w" in z:
        return z["w"]
    ids, wt = z[ids_key], z["weights"]
    return np.where(ids >= 0, wt[np.clip(ids, 0, None)], 0.0).astype(np.float32)


def emb_base(z, ids_key="ids"):
    return emb_sequential(table(z), z[ids_key], seq_weights(z, ids_key))


def emb(z, ids_key="ids"):
    return (emb_base(z, ids_key).view(np.int32) + z["emb__resid"]).view(np.float32)


def g8_inputs(z):
    """make_goldens_latent.py matrix_case: rng 82 -> ids, audio, visual,
    amask, vmask, lat (in that order)."""
    B, T, A, Vd, V = 24, 10, int(z["A"]), int(z["Vd"]), int(z["V"])
    rng = np.random.default_rng(82)
    ids = rng.integers(1, V, size=(B, T)).astype(np.int64)
    ids[:, :2] = 0
    aud = rng.standard_normal((B, T, A)).astype(np.float32)
    vis = rng.standard_normal((B, T, Vd)).astype(np.float32)
    am = (rng.random((B, T, A)) > 0.1).astype(np.float32)
    vm = (rng.random((B, T, Vd)) > 0.1).astype(np.float32)
    lat = (0.5 * rng.standard_normal((B, 300))).astype(np.float32)
    return {"ids": ids, "audio": aud, "visual": vis, "amask": am, "vmask": vm, "lat": lat}


def g7_word_inputs(z):
    """make_goldens_latent.py word_case: table seed 71, rng 72 -> ids, lens,
    lat, up."""
    V, B, Lt = int(z["V"]), 48, 20
    E = table({"V": V, "table_seed": z["table_seed"], "table_checksum": z["table_checksum"]})
    rng = np.random.default_rng(72)
    ids = rng.integers(1, V, size=(B, Lt)).astype(np.int64)
    lens = rng.integers(3, Lt + 1, size=B)
    ids[np.arange(Lt)[None, :] >= lens[:, None]] = 0
    lat = (0.5 * rng.standard_normal((B, 300)) + 0.3 * E[ids[:, 0]]).astype(np.float32)
    up = rng.standard_normal(B).astype(np.float32)
    return {"ids": ids, "lat": lat, "up": up}


def g7_gauss_inputs(z, B, T, F, seed):
    """make_goldens_latent.py gauss_case."""
    rng = np.random.default_rng(seed)
    mu = rng.standard_normal((B, F)).astype(np.float32)
    sg = np.exp(0.3 * rng.standard_normal((B, F))).astype(np.float32)
    x = rng.standard_normal((B, T, F)).astype(np.float32)
    m = (rng.random((B, T, F)) > 0.2).astype(np.float32)
    up = rng.standard_normal(B).astype(np.float32)
    return {"mu": mu, "sigma": sg, "x": x, "mask": m, "up": up}


def g5_step_inputs(z):
    """make_goldens.py G5: torch.manual_seed(0) then the reference model's two
    nn.Linear layers (sentiment_model.py:33-34, in construction order); x from
    rng 15, y from rng 16."""
    import torch

    torch.manual_seed(0)
    h1 = torch.nn.Linear(300, 100)
    out = torch.nn.Linear(100, 1)
    x = np.random.default_rng(15).standard_normal((32, 300)).astype(np.float32)
    y = np.random.default_rng(16).uniform(-3, 3, 32).astype(np.float32)
    return {"x": x, "y": y, "w1": h1.weight.detach().numpy().copy(), "b1": h1.bias.detach().numpy().copy(),
            "w2": out.weight.detach().numpy().copy(), "b2": out.bias.detach().numpy().copy()}


GAUSS = {"g7_gauss": (16, 12, 37, 91), "g7_gauss_b1": (1, 12, 37, 92)}


def recipe(name):
    """fixture name -> recipe(z) -> {key: array}, or None."""
    if name in ("g1_pom_valid", "g1_pom_test", "g2_mosi", "g3_gap", "g3b_npc2"):
        return lambda z: {"emb": emb(z)}
    if name == "g1c_seq2weight":
        return lambda z: {"emb": emb(z, "seq")}
    if name == "g8_matrix":
        return g8_inputs
    if name in ("g7_word", "g7_word_ids"):
        return g7_word_inputs
    if name in GAUSS:
        return lambda z: g7_gauss_inputs(z, *GAUSS[name])
    if name == "g5_senti_step":
        return g5_step_inputs
    return None
