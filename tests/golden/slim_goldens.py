#!/usr/bin/env python3
"""Shrink the committed fixtures without losing what the tests check (r03).

The fixtures were recorded from the reference by make_goldens*.py (which
import /root/reference); this script rewrites them in place, needing only
the fixtures themselves, and is idempotent.  Every transformation is either
lossless (checked bit for bit here) or keeps a sample that the tests compare
the same way:

* g1_pom_* / g2_mosi / g3_gap / g3b_npc2: the f64 removal output `out`
  [n, 300] is stored as its rank-npc correction `out_coef` = X.dot(pc.T)
  (X = emb in f64), so out = X - out_coef * pc (npc = 1: elementwise, bit for
  bit anywhere) or X - out_coef.dot(pc) (npc = 2: bit for bit with this
  host's BLAS, to the rounding of a 2-term dot elsewhere) -- the reference's
  own expressions (sif_functions.py:77-80), rebuilt by tests/conftest.py's
  loader (asserted below).
* g1_pom_*: the seq2weight output `w` = f32(weights[ids]) for ids >= 0, else
  0 (sif_functions.py:8-15, elementwise) is rebuilt and checked against the
  sha256 of the reference's bytes, recorded here.
* g5_senti_train: the latents (rng = default_rng(17), standard normal) are
  regenerated from the seed and checked by checksum.
* g5_senti_step: nw1 = w1 - 0.1 gw1 in f32 (torch SGD), rebuilt bit for bit.
* g4_mmb2_syn: calc_qm_audio / calc_qs_audio dropped (no test reads them;
  g4_mmb2_mosi keeps the calc_weights fixture).
* g8_matrix: every parameter gradient larger than 50 KB keeps every 16th row
  (larger than 20 KB: every 4th) plus the whole tensor's max |.| (the per-tensor scale of the gradient check)
  -- the test compares those rows against that scale.
* g9_cli_*: the pre / post embeddings keep every 8th row (`rows`); the test
  compares those rows with the same row-relative bars.
* seeded inputs (g7, g8, g5_senti_step: numpy default_rng / torch CPU
  generator streams) and the a2 rows `emb` (g1*, g2, g3, g3b: the BLAS-free
  f32 accumulation of tests/golden/regen.py + a stored int32 ULP residual)
  are rebuilt by regen.py's recipes, checked here bit for bit and by the
  loader against the recorded `<key>__sha256`.

    python tests/golden/slim_goldens.py
"""
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def load(name):
    return dict(np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False))


def save(name, d):
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)


def rebuild_out(z):
    X = z["emb"].astype(np.float64)
    pc = z["pc"]
    c = z["out_coef"]
    return X - c * pc if pc.shape[0] == 1 else X - c.dot(pc)


def slim_removal(name):
    z = load(name)
    if "out" not in z:
        return
    X = z["emb"].astype(np.float64)
    z["out_coef"] = X.dot(z["pc"].transpose())
    rec = rebuild_out(z)
    assert np.array_equal(rec, z["out"]), name
    del z["out"]
    save(name, z)


def rebuild_w(z):
    ids, wt = z["ids"], z["weights"]
    return np.where(ids >= 0, wt[np.clip(ids, 0, None)], 0.0).astype(np.float32)


def sha(a) -> str:
    import hashlib

    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def slim_seq2weight(name):
    z = load(name)
    if "w" not in z:
        return
    assert np.array_equal(rebuild_w(z), z["w"]), name
    z["w_sha256"] = np.array(sha(z["w"]))
    del z["w"]
    save(name, z)


def latents_17():
    rng = np.random.default_rng(17)
    return [rng.standard_normal((n, 300)).astype(np.float32) for n in (200, 50, 70)]


def slim_senti_train():
    z = load("g5_senti_train")
    if "lat_train" not in z:
        return
    lat = latents_17()
    for k, l in zip(("lat_train", "lat_valid", "lat_test"), lat):
        assert np.array_equal(l, z[k]), k
        z[k + "_checksum"] = np.float64(np.asarray(z[k], np.float64).sum())
        del z[k]
    z["lat_seed"] = np.int64(17)
    save("g5_senti_train", z)


def rebuild_nw1(z):
    w1, gw1 = torch.tensor(z["w1"]), torch.tensor(z["gw1"])
    return w1.add(gw1, alpha=-float(z["nw1_lr"])).numpy()


def slim_senti_step():
    z = load("g5_senti_step")
    if "nw1" not in z:
        return
    z["nw1_lr"] = np.float64(0.1)
    if np.array_equal(rebuild_nw1(z), z["nw1"]):
        del z["nw1"]
        save("g5_senti_step", z)


def slim_g4_syn():
    z = load("g4_mmb2_syn")
    if "calc_qm_audio" in z:
        del z["calc_qm_audio"], z["calc_qs_audio"]
        save("g4_mmb2_syn", z)


def slim_g8():
    z = load("g8_matrix")
    changed = False
    for k in list(z):
        v = z[k]
        if (k.startswith("grad_") and not k.endswith(("__rows", "__absmax")) and v.nbytes > 20_000
                and k + "__rows" not in z):
            rows = np.arange(0, v.shape[0], 16 if v.nbytes > 50_000 else 4)
            z[k + "__absmax"] = np.float64(np.abs(v).max())
            z[k + "__rows"] = rows
            z[k] = v[rows]
            changed = True
    if changed:
        save("g8_matrix", z)


def slim_g9(variant):
    name = f"g9_cli_{variant}"
    z = load(name)
    if "rows" in z:
        return
    rows = np.arange(0, z["pre"].shape[0], 8)
    z["rows"] = rows
    z["pre"] = z["pre"][rows]
    z["post"] = z["post"][rows]
    save(name, z)


class _View(dict):
    """A fixture dict seen through the loader: `w` rebuilt if dropped."""

    def __getitem__(self, k):
        if k == "w" and not dict.__contains__(self, "w") and dict.__contains__(self, "w_sha256"):
            return rebuild_w(self)
        return dict.__getitem__(self, k)

    def __contains__(self, k):
        return dict.__contains__(self, k) or (k == "w" and dict.__contains__(self, "w_sha256"))


def slim_regen(name):
    """Drop every array tests/golden/regen.py's recipe rebuilds bit for bit
    (the a2 rows via their int32 ULP residual), recording its sha256."""
    import regen

    z = _View(load(name))
    if "emb" in z and "emb__resid" not in z:
        base = regen.emb_base(z, "seq" if name == "g1c_seq2weight" else "ids")
        z["emb__resid"] = z["emb"].view(np.int32) - base.view(np.int32)
    got = regen.recipe(name)(z)
    changed = False
    for k, a in got.items():
        if dict.__contains__(z, k) and z[k].nbytes > 4096:
            assert a.dtype == z[k].dtype and np.array_equal(a.view(np.uint8), z[k].view(np.uint8)), (name, k)
            z[k + "__sha256"] = np.array(regen.sha(z[k]))
            del z[k]
            changed = True
    if changed:
        save(name, dict(z))


def main():
    for n in ("g1_pom_valid", "g1_pom_test", "g2_mosi", "g3_gap", "g3b_npc2"):
        slim_removal(n)
    for n in ("g1_pom_valid", "g1_pom_test"):
        slim_seq2weight(n)
    slim_senti_train()
    slim_senti_step()
    slim_g4_syn()
    slim_g8()
    for v in ("e2e_sgd_ln", "e2e_adam_bn", "mmb1_e2e", "opt_sgd_ln", "pom_e2e"):
        slim_g9(v)
    for n in ("g1_pom_valid", "g1_pom_test", "g2_mosi", "g3_gap", "g3b_npc2", "g1c_seq2weight",
              "g8_matrix", "g7_word", "g7_word_ids", "g7_gauss", "g7_gauss_b1", "g5_senti_step"):
        slim_regen(n)
    total = sum(os.path.getsize(os.path.join(HERE, f)) for f in os.listdir(HERE)
                if f.endswith((".npz", ".json")))
    print(f"fixtures: {total / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
