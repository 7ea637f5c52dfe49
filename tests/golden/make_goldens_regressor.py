"""Full-size regressor fixtures (BASELINE configs[4]) made by running the REFERENCE.

Run in the build container only (needs /root/reference, read-only):

    python tests/golden/make_goldens_regressor.py

It calls the reference's own `sentiment_model.train_sentiment_for_latents`
(`/root/reference/sentiment_model.py:165-265`) on MOSI-sized splits
(1284 / 229 / 686 rows, SURVEY.md §8 shapes) for the configs' 400 epochs
(`configs/make_configs.py:25`), H = 100, lr 0.1, batch 32:

  g5_full          early_stopping False (the plain SGD loop, :98-127)
  g5_full_es       early_stopping True with a model_save_path: the patience /
                   trials / lr-decay / best-model reload branch (:132-160) and
                   the "evaluate the un-reloaded model" quirk (:243-250)

Only data is stored: the latents and labels are regenerated from the seed by
`latents_and_labels()` below (also imported by the GPU test) and checked by
checksum; the fixture holds the recorded loss curves, the final parameters,
the metric dicts, the files the run wrote, and which early-stopping events
fired (parsed from the reference's own prints).
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
SIZES = (1284, 229, 686)
# (fixture, early_stopping, seed, label noise): with noise 1.5 the ES run reloads
# the best model twice (lr decayed each time) and then stops early at epoch 330
CASES = (("g5_full", False, 4242, 0.9), ("g5_full_es", True, 4343, 1.5))


def latents_and_labels(seed: int, sizes=SIZES, noise: float = 0.9):
    """Seeded MOSI-shaped latents (unit-norm-ish rows like SIF output) and
    labels in [-3, 3] (MOSI's range) that a 300->100->1 net can fit but,
    with label noise, overfits -- so validation loss turns up and the
    early-stopping branch is exercised."""
    rng = np.random.default_rng(seed)
    lat = [(rng.standard_normal((n, 300)) / np.sqrt(300)).astype(np.float32) for n in sizes]
    wproj = rng.standard_normal(300).astype(np.float32) * np.float32(2.0)
    wq = rng.standard_normal(300).astype(np.float32) * np.float32(2.0)
    labels = [np.clip(l @ wproj + np.abs(l @ wq) - 1.0 + noise * rng.standard_normal(l.shape[0]),
                      -3, 3).astype(np.float32) for l in lat]
    return lat, labels


def checksum(a) -> float:
    return float(np.asarray(a, dtype=np.float64).sum())


def run_reference(R_sm, args, lat, labels, seed, save_dir):
    import torch

    captured, metrics = {}, []
    orig, orig_fl = R_sm.train_sentiment, R_sm.full_loss

    def spy(*a, **k):
        tl, vl = orig(*a, **k)
        captured["train"] = [float(t) for t in tl]
        captured["valid"] = [float(t) for t in vl]
        captured["model"] = {kk: v.detach().clone() for kk, v in a[1].state_dict().items()}
        return tl, vl

    def spy_fl(p, y):
        r = orig_fl(p, y)
        metrics.append(r)
        return r

    R_sm.train_sentiment, R_sm.full_loss = spy, spy_fl
    buf = io.StringIO()
    try:
        torch.manual_seed(seed)
        with contextlib.redirect_stdout(buf):
            R_sm.train_sentiment_for_latents(args, tuple(torch.tensor(l) for l in lat),
                                              tuple(labels), torch.device("cpu"),
                                              model_save_path=save_dir)
    finally:
        R_sm.train_sentiment, R_sm.full_loss = orig, orig_fl
    log = buf.getvalue().splitlines()
    events = {"reloads": sum("reloading model and decaying" in s for s in log),
              "early_stop": any(s.strip() == "early stopping..." for s in log),
              "patience_lines": sum(s.startswith("patience ") for s in log)}
    return captured, metrics, events


def main():
    sys.path.insert(0, REF)
    sys.modules.setdefault("h5py", types.ModuleType("h5py"))
    import sentiment_model as R_sm  # noqa: E402

    for name, es, seed, noise in CASES:
        lat, labels = latents_and_labels(seed, noise=noise)
        args = {"sentiment_hidden_size": 100, "n_sentiment_epochs": 400, "sentiment_lr": 0.1,
                "early_stopping": es, "dataset": "mosi", "lr_decay": 0.5}
        with tempfile.TemporaryDirectory() as d:
            cap, metrics, events = run_reference(R_sm, args, lat, labels, seed, d)
            files = sorted(os.listdir(d))
            text = {}
            for f in ("senti_train_loss.txt", "senti_valid_loss.txt", "test_acc_before.txt",
                      "test_acc_after.txt"):
                with open(os.path.join(d, f)) as fh:
                    text[f] = fh.read()
        print(name, events, "epochs run:", len(cap["train"]), "validations:", len(cap["valid"]))
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"), seed=np.int64(seed),
            lat_checksums=np.array([checksum(l) for l in lat]),
            label_checksums=np.array([checksum(l) for l in labels]),
            train_losses=np.array(cap["train"]), valid_losses=np.array(cap["valid"]),
            **{"final_" + k.replace(".", "_"): v.numpy() for k, v in cap["model"].items()})
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump({"args": args, "noise": noise, "before": metrics[0], "after": metrics[1], "events": events,
                       "files": files, "text_files": text}, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
