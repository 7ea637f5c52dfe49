"""CPU: pin the oracle (oracle/) to the golden fixtures made by running the reference.

The reference ships no tests; tests/golden/make_goldens.py ran
the reference's own functions in the build container and recorded inputs and
outputs.  These tests check that the CPU restatement reproduces them, so the
oracle can stand in for the reference on the GPU box.
"""
import json
import os

import numpy as np
import pytest

import synth
from oracle import mmb2_oracle as M
from oracle import sif_oracle as O

SIF_CASES = ["g1_pom_valid", "g1_pom_test", "g2_mosi", "g3_gap"]


def regen_table(z):
    E = synth.word_table(int(z["V"]), int(z["D"]), seed=int(z["table_seed"]),
                         common=float(z["common"]))
    assert float(np.asarray(E, np.float64).sum()) == float(z["table_checksum"])
    return E


@pytest.mark.parametrize("case", SIF_CASES)
def test_seq2weight_bit_exact(golden, case):
    z = golden(case)
    w = O.seq2weight(z["ids"], np.ones(z["ids"].shape), z["weights"])
    assert w.dtype == np.float32
    assert np.array_equal(w, z["w"])


def test_seq2weight_mask_negative(golden):
    z = golden("g1c_seq2weight")
    assert np.array_equal(O.seq2weight(z["seq"], z["mask"], z["weights"]), z["w"])
    assert np.array_equal(O.seq2weight_loop(z["seq"], z["mask"], z["weights"]), z["w"])


@pytest.mark.parametrize("case", SIF_CASES)
def test_weighted_average(golden, case):
    z = golden(case)
    E = regen_table(z)
    emb = O.get_weighted_average(E, z["ids"], z["w"])
    assert emb.dtype == np.float64
    assert np.array_equal(emb, z["emb"].astype(np.float64))


@pytest.mark.parametrize("case", SIF_CASES + ["g3b_npc2"])
def test_compute_pc_matches_sklearn_run(golden, case):
    z = golden(case)
    X = z["emb"].astype(np.float64)
    npc = z["pc"].shape[0]
    assert np.array_equal(O.compute_pc(X, npc), z["pc"])


@pytest.mark.parametrize("case", SIF_CASES)
def test_sif_embedding_end_to_end(golden, case):
    z = golden(case)
    E = regen_table(z)
    out = O.get_sentence_embeddings(E, z["weights"], z["ids"])
    assert np.array_equal(out, z["out"])


def test_remove_pc_npc2(golden):
    z = golden("g3b_npc2")
    # the pc agrees bit for bit (test above); the final BLAS dot may sum in a
    # different order for a differently strided pc, so allow f64 rounding here
    got = O.remove_pc(z["emb"].astype(np.float64), 2)
    assert M.row_rel_err(got, z["out"]) < 1e-13


def test_randomized_restatement_equals_sklearn():
    """The restatement is the third-party algorithm (sklearn 1.7.2 here)."""
    sk = pytest.importorskip("sklearn.decomposition")
    rng = np.random.default_rng(0)
    for shape in [(50, 300), (400, 300), (301, 300)]:
        X = rng.standard_normal(shape) + 0.5
        svd = sk.TruncatedSVD(n_components=1, n_iter=7, random_state=0).fit(X)
        assert np.array_equal(O.compute_pc(X, 1), svd.components_)


def test_gap_case_is_not_the_exact_svd(golden):
    """With s1/s2 ~ 1.06 the randomized PC is NOT the exact top singular vector
    — the oracle (and the device solver) must reproduce the randomized one."""
    z = golden("g3_gap")
    assert float(z["s1_s2"]) < 1.2
    exact = O.exact_top_pc(z["emb"].astype(np.float64))
    assert np.abs(exact - z["pc"]).max() > 1e-3


def _mmb2_inputs(z, dtype=np.float64):
    import torch
    import models

    A, Vd, V = int(z["A"]), int(z["Vd"]), int(z["V"])
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None, frozen_weights=True)
    sums = np.array([float(np.asarray(p.detach().numpy(), np.float64).sum())
                     for p in gen.state_dict().values()])
    assert np.array_equal(sums, z["param_checksums"])
    E = synth.word_table(V, 300, seed=int(z["table_seed"]))
    ids = z["ids"]
    N, T = ids.shape
    pe = float(z["pad_frac"])
    audio = synth.frames(N, T, A, seed=int(z["audio_seed"]), pad_frac=pe)
    visual = synth.frames(N, T, Vd, seed=int(z["visual_seed"]), pad_frac=pe)
    assert float(np.asarray(audio, np.float64).sum()) == float(z["audio_checksum"])
    wt32 = z["weights"].astype(np.float32)
    sw = np.where(ids >= 0, wt32[ids], 0).astype(np.float32)
    text = E[ids]
    return gen, E, ids, audio, visual, sw, text


@pytest.mark.parametrize("case", ["g4_mmb2_mosi", "g4_mmb2_syn"])
def test_mmb2_oracle(golden, case):
    z = golden(case)
    gen, E, ids, audio, visual, sw, text = _mmb2_inputs(z)
    data = M.concat_inputs(text, audio, visual)
    params = M.params_from_module(gen)
    cs64 = M.estimate_embedding_overall_gpu2(data, params, sw, text, dtype=np.float64)
    assert M.row_rel_err(cs64, z["cs_f64"]) < 1e-12
    cs32 = M.estimate_embedding_overall_gpu2(data, params, sw, text, dtype=np.float32)
    assert M.row_rel_err(cs32, z["cs_f32"]) < 2e-6
    # the reference's own fp32 run sits well inside the 1e-5 bar of its f64 run
    assert M.row_rel_err(z["cs_f32"], z["cs_f64"]) < 1e-5


def test_calc_weights_oracle(golden):
    z = golden("g4_mmb2_mosi")
    gen, E, ids, audio, visual, sw, text = _mmb2_inputs(z)
    b = gen.embed2out["audio"]["mu"].bias.detach().numpy()
    ls = gen.embed2out["audio"]["log_sigma"].bias.detach().numpy()
    qm, qs = M.calc_weights(audio[:4], b, ls)
    np.testing.assert_allclose(qm, z["calc_qm_audio"], rtol=2e-6, atol=1e-6)
    np.testing.assert_allclose(qs, z["calc_qs_audio"], rtol=2e-6, atol=1e-5)


def test_metrics_match_reference(golden):
    """losses.py metrics (host numpy/sklearn by design) vs the reference run."""
    import losses as MO

    z = golden("g6_metrics_inputs")
    with open(os.path.join(os.path.dirname(__file__), "golden", "g6_metrics.json")) as f:
        ref = json.load(f)
    got = {"full": MO.full_loss(z["pred"], z["y"], verbose=False),
           "pom": MO.pom_loss(z["pred_pom"], z["y_pom"], verbose=False),
           "iemocap": MO.iemocap_loss(z["pred_iemocap"], z["y_iemocap"], verbose=False)}
    assert json.loads(json.dumps(got)) == ref


def test_sliced_gram_restatement_meets_pc_bar(golden):
    """The int8-digit Gram (oracle.sif_oracle.sliced_gram, the device
    mmb_gram_i8's arithmetic): within 2e-10 of the exact Gram and its PC within
    1e-9 of the reference TruncatedSVD component on every golden split."""
    for case in ("g2_mosi", "g3_gap", "g3b_npc2"):
        z = golden(case)
        X = z["emb"].astype(np.float64)
        G = X.T @ X
        Gs = O.sliced_gram(z["emb"])
        assert np.abs(Gs - G).max() <= 2e-10 * np.abs(G).max()
        npc = z["pc"].shape[0]
        z0 = np.random.RandomState(0).normal(size=(X.shape[1], npc + 10))
        pc = O.pc_from_gram(Gs, z0, npc, False)
        assert np.abs(pc - z["pc"]).max() < 1e-9, case


@pytest.mark.parametrize("split", ["valid", "test"])
def test_real_pom_split_end_to_end(golden, split):
    """g11: the reference's get_sentence_embeddings on a WHOLE real POM split
    (pom_valid_ids 100 x 1089 / pom_test_ids 203 x 1357, real weights, its
    own PC: simplesif.py:296-311), reproduced by the oracle -- PC bit for bit
    (the transposed randomized-SVD branch, n < 300) and the recorded rows."""
    z = golden("g11_pom_splits")
    E = synth.word_table(int(z["V"]), 300, seed=int(z["table_seed"]))
    assert float(np.asarray(E, np.float64).sum()) == float(z["table_checksum"])
    ids = z[f"{split}_ids"].astype(np.int64)
    w = O.seq2weight(ids, np.ones(ids.shape), z["weights"])
    x = O.get_weighted_average(E, ids, w)
    assert np.array_equal(O.compute_pc(x, 1), z[f"{split}_pc"])
    out = O.get_sentence_embeddings(E, z["weights"], ids)
    assert np.array_equal(out[::int(z["row_step"])], z[f"{split}_out_rows"])
