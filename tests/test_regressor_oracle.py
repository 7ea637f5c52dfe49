"""CPU: the regressor restatement (oracle/regressor_oracle.py) against the reference's runs.

Pins the oracle the GPU regressor tests and bench.py's regressor cpu_baseline
rely on: the 20-epoch g5_senti_train run exactly, the full-size (1284 / 229 /
686, 400 epochs) g5_full run over its first 20 epochs, and the full-size
early-stopping run g5_full_es end to end (two best-model reloads with lr
decay at epochs 100 and 200, then the early stop at epoch 300,
sentiment_model.py:132-160) -- bit for bit: the oracle is the reference's
loop in the same torch CPU arithmetic.
"""
import importlib.util
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from losses import full_loss
from oracle import regressor_oracle as R


def _gen():
    spec = importlib.util.spec_from_file_location(
        "make_goldens_regressor", os.path.join(GOLDEN, "make_goldens_regressor.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def full_case(name):
    """(args, latents, labels, fixture, meta) of a g5_full* fixture, inputs
    regenerated from the recorded seed and checked by checksum."""
    g = _gen()
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        meta = json.load(f)
    lat, lab = g.latents_and_labels(int(z["seed"]), noise=meta["noise"],
                                    flip_valid=meta["flip_valid"])
    assert np.allclose([g.checksum(l) for l in lat], z["lat_checksums"], rtol=0, atol=1e-9)
    assert np.allclose([g.checksum(l) for l in lab], z["label_checksums"], rtol=0, atol=1e-9)
    return dict(meta["args"]), lat, lab, z, meta


def _quiet(fn, *a):
    import contextlib
    import io

    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a)


def test_oracle_matches_reference_20_epochs(golden):
    z = golden("g5_senti_train")
    with open(os.path.join(GOLDEN, "g5_senti_train_metrics.json")) as f:
        ref = json.load(f)
    args = {"sentiment_hidden_size": 100, "n_sentiment_epochs": 20, "sentiment_lr": 0.1,
            "early_stopping": False, "dataset": "mosi", "lr_decay": 0.5}
    torch.manual_seed(int(z["seed"]))
    r = R.train_for_latents(args, (z["lat_train"], z["lat_valid"], z["lat_test"]),
                            (z["y_train"], z["y_valid"], z["y_test"]))
    assert np.array_equal(r["train_losses"], z["train_losses"])
    assert np.array_equal(r["valid_losses"], z["valid_losses"])
    for k, v in r["state"].items():
        assert np.array_equal(v.numpy(), z["final_" + k.replace(".", "_")])
    after = _quiet(full_loss, *r["after"])
    assert after["mae"] == pytest.approx(ref["after"]["mae"], abs=1e-12)
    assert after["accuracy"] == ref["after"]["accuracy"]


def test_oracle_matches_full_size_run_prefix():
    """configs[4] shape, first 20 of the 400 epochs (the same RNG stream)."""
    args, lat, lab, z, _ = full_case("g5_full")
    args["n_sentiment_epochs"] = 20
    torch.manual_seed(int(z["seed"]))
    r = R.train_for_latents(args, lat, lab)
    assert np.array_equal(r["train_losses"], z["train_losses"][:20])
    assert np.array_equal(r["valid_losses"], z["valid_losses"][:2])


@pytest.mark.slow
def test_oracle_matches_full_size_early_stopping_run():
    args, lat, lab, z, meta = full_case("g5_full_es")
    torch.manual_seed(int(z["seed"]))
    r = R.train_for_latents(args, lat, lab)
    assert r["events"] == {"reloads": 2, "early_stop": True}
    assert meta["events"]["reloads"] == 2 and meta["events"]["early_stop"]
    assert np.array_equal(r["train_losses"], z["train_losses"])
    assert np.array_equal(r["valid_losses"], z["valid_losses"])
    for k, v in r["state"].items():
        assert np.array_equal(v.numpy(), z["final_" + k.replace(".", "_")])
    after = _quiet(full_loss, *r["after"])
    assert after["mae"] == pytest.approx(meta["after"]["mae"], abs=1e-12)
    assert after["corr"] == pytest.approx(meta["after"]["corr"], abs=1e-12)
