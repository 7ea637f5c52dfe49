"""CPU: pin the latent-objective oracle and the data-preparation mirror to the
reference's own outputs (tests/golden/make_goldens_latent.py), and check the
CLI surface that needs no GPU (argument parsing, config handling)."""
import copy
import json
import os

import numpy as np
import pytest
import torch

import synth
from oracle import latent_oracle as LO

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def word_inputs(z):
    E = synth.word_table(int(z["V"]), 300, seed=int(z["table_seed"]))
    assert float(np.asarray(E, np.float64).sum()) == float(z["table_checksum"])
    wts = torch.tensor(synth.sif_weights(int(z["V"])), dtype=torch.float32)
    return torch.tensor(E), wts, torch.tensor(z["ids"])


def test_oracle_word_angular2(golden):
    z = golden("g7_word")
    table, wts, ids = word_inputs(z)
    x = torch.tensor(z["lat"], requires_grad=True)
    mask = (ids != 0).float()[:, :, None].expand(*ids.shape, 300)
    lp = LO.word_log_prob_angular2(x, table, wts[ids], table[ids], mask, 1e-3)
    (lp * torch.tensor(z["up"])).sum().backward()
    np.testing.assert_allclose(lp.detach().numpy(), z["lp"], rtol=2e-6, atol=1e-5)
    np.testing.assert_allclose(x.grad.numpy(), z["dlat"], rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("case", ["g7_gauss", "g7_gauss_b1"])
def test_oracle_normal(golden, case):
    z = golden(case)
    mu = torch.tensor(z["mu"], requires_grad=True)
    sg = torch.tensor(z["sigma"], requires_grad=True)
    lp = LO.normal_log_prob(mu[:, None], sg[:, None], torch.tensor(z["x"]), torch.tensor(z["mask"]))
    up = torch.tensor(z["up"])
    (lp * (up[:1] if lp.dim() == 0 else up)).sum().backward()
    assert lp.shape == z["lp"].shape  # B = 1: the squeeze quirk makes a scalar
    np.testing.assert_allclose(lp.detach().numpy(), z["lp"], rtol=1e-6)
    np.testing.assert_allclose(mu.grad.numpy(), z["dmu"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(sg.grad.numpy(), z["dsigma"], rtol=1e-5, atol=1e-6)


def test_utils_normalize_and_positions(golden):
    import utils

    z = golden("g10_utils")
    _, _, (tr, _, _) = synth.mm_splits(seed=11, sizes=(40, 8, 8), T=9, V=50, A_raw=7, Vd_raw=5)
    d, m = utils.normalize_data(copy.deepcopy(tr))
    assert np.array_equal(d["covarep"], z["covarep"])  # constant feature dropped, +min quirk
    assert np.array_equal(d["facet"], z["facet"])
    assert np.array_equal(m["covarep"], z["cov_mask"]) and np.array_equal(m["facet"], z["fac_mask"])
    pe2 = utils.add_positional_embeddings({"pos_embed_dim": 2}, d["covarep"])
    pe4 = utils.add_positional_embeddings({"pos_embed_dim": 4}, d["facet"])
    assert pe2.dtype == z["pe2"].dtype and np.array_equal(pe2, z["pe2"])
    assert np.array_equal(pe4, z["pe4"])
    # the utterance-axis quirk: only utterances 0..pe-1 carry sin/cos
    assert np.array_equal(pe4[5, :, -4:], np.tile(np.arange(9, dtype=np.float32)[:, None], (1, 4)))


def test_utils_npz_twin_roundtrip(tmp_path, monkeypatch):
    import utils

    w2i, E, splits = synth.mm_splits(seed=3, sizes=(6, 4, 4), T=5, V=20, A_raw=4, Vd_raw=3)
    monkeypatch.chdir(tmp_path)
    os.makedirs("data")
    utils.save_splits_npz("data/mosi_data.npz", splits)
    got = utils._read_splits("data/mosi_data.h5", utils.H5_KEYS["mosi"])
    for a, b in zip(got, splits):
        for k in utils.H5_KEYS["mosi"]:
            assert np.array_equal(a[k], b[k])


def test_cli_arguments(tmp_path):
    import simplesif

    cfg = {"sentiment_hidden_size": 150, "lr": 1e-4, "sentiment_lr": 0.01, "seq_len": 20,
           "word_sim_metric": "angular", "n_epochs": 100, "freeze_weights": False,
           "n_sentiment_epochs": 400, "word_loss_weight": 0.002, "likelihood_weight": 0.0001,
           "pos_embed_dim": 4, "e2e": True, "norm": "batch_norm", "optimizer": "adam",
           "config_num": 7}
    p = tmp_path / "config_7.json"
    p.write_text(json.dumps(cfg))
    a = simplesif.parse_arguments([str(p), "mosi", "--e2e", "n", "--pos_embed_dim", "2",
                                   "--sentiment_epochs", "5", "--likelihood_weight", "0.5"])
    assert a["e2e"] is False and a["pos_embed_dim"] == 2 and a["n_sentiment_epochs"] == 5
    assert a["likelihood_weight"] == 0.0001  # the flag is parsed but the config wins (:219-227)
    assert a["batch_size"] == 64 and a["optimizer"] == "adam" and a["config_num"] == 7


def test_cli_golden_files_listed():
    """Every CLI golden records the run tree the reference wrote."""
    for v in ("e2e_sgd_ln", "e2e_adam_bn", "opt_sgd_ln", "mmb1_e2e", "pom_e2e"):
        j = json.load(open(os.path.join(GOLDEN, f"g9_cli_{v}.json")))
        assert {"config.json", "pre/embed.bin", "post/embed.bin", "embed_loss.txt",
                "post/senti.bin"} <= set(j["files"])


def test_config_grid_seeded(tmp_path):
    import importlib.util

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("mk", os.path.join(root, "configs", "make_configs.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    a = mk.main(["--seed", "0", "--out", str(tmp_path / "g1")])
    b = mk.main(["--seed", "0", "--out", str(tmp_path / "g2")])
    assert len(a) == 512 and a == b  # 2^9 points (make_configs.py:16-31), seeded order
    assert len({json.dumps(c, sort_keys=True) for c in a}) == 512
    pinned = json.load(open(os.path.join(root, "configs", "multimodal_search", "config_0.json")))
    assert pinned == a[0]
    import simplesif

    args = simplesif.parse_arguments([os.path.join(root, "configs", "multimodal_search",
                                                    "config_0.json"), "mosi"])
    assert args["config_num"] == 0 and args["e2e"] is True
