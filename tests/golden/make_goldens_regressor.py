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
# (fixture, early_stopping, seed, label noise, validation labels flipped).
# g5_full_es flips the validation labels' sign: every SGD step that fits the
# training split moves the validation loss up, so after the first validation
# none is better -- 10 bad validations (epoch 100) reload the epoch-0
# checkpoint with lr * 0.5, again at epoch 200, and the third trial stops at
# epoch 300.  The margins between validations are wide, so these events do
# not depend on rounding (the plain run's loss curve does, see ENVELOPE).
CASES = (("g5_full", False, 4242, 0.9, False), ("g5_full_es", True, 4343, 0.9, True))


def latents_and_labels(seed: int, sizes=SIZES, noise: float = 0.9, flip_valid: bool = False):
    """Seeded MOSI-shaped latents (unit-norm-ish rows like SIF output) and
    labels in [-3, 3] (MOSI's range) that a 300->100->1 net can fit, with
    label noise (it overfits)."""
    rng = np.random.default_rng(seed)
    lat = [(rng.standard_normal((n, 300)) / np.sqrt(300)).astype(np.float32) for n in sizes]
    wproj = rng.standard_normal(300).astype(np.float32) * np.float32(2.0)
    wq = rng.standard_normal(300).astype(np.float32) * np.float32(2.0)
    labels = [np.clip(l @ wproj + np.abs(l @ wq) - 1.0 + noise * rng.standard_normal(l.shape[0]),
                      -3, 3).astype(np.float32) for l in lat]
    if flip_valid:
        labels[1] = -labels[1]
    return lat, labels


# The loss curve of 16,400 fp32 SGD steps on an L1 loss is sensitive to
# rounding: every residual that crosses 0 flips its gradient.  Each fixture
# therefore also records the SAME reference function run (a) in float64 and
# (b) in float32 on latents nudged by one ulp -- two rounding-level
# perturbations of the reference itself.  Their distance from the recorded
# run is the envelope a different-but-correct fp32 implementation (the GPU's
# summation order) is held to after the first epochs.
ENVELOPE = ("f64", "ulp")


def checksum(a) -> float:
    return float(np.asarray(a, dtype=np.float64).sum())


def run_reference(R_sm, args, lat, labels, seed, save_dir, dtype=None):
    import torch

    if dtype is not None:
        torch.set_default_dtype(dtype)

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
        torch.set_default_dtype(torch.float32)
    log = buf.getvalue().splitlines()
    events = {"reloads": sum("reloading model and decaying" in s for s in log),
              "early_stop": any(s.strip() == "early stopping..." for s in log),
              "patience_lines": sum(s.startswith("patience ") for s in log)}
    return captured, metrics, events


def main():
    sys.path.insert(0, REF)
    sys.modules.setdefault("h5py", types.ModuleType("h5py"))
    import sentiment_model as R_sm  # noqa: E402

    import torch

    for name, es, seed, noise, flip in CASES:
        lat, labels = latents_and_labels(seed, noise=noise, flip_valid=flip)
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
        env = {}
        for kind in ENVELOPE:
            if kind == "f64":
                lat_k, dt = [l.astype(np.float64) for l in lat], torch.float64
            else:
                lat_k, dt = [np.nextafter(l, np.float32(np.inf)) for l in lat], None
            with tempfile.TemporaryDirectory() as d:
                c2, m2, e2 = run_reference(R_sm, args, lat_k, labels, seed, d, dtype=dt)
            env[kind] = {"train_losses": c2["train"], "valid_losses": c2["valid"],
                         "after": m2[1], "events": e2}
            tl = np.array(c2["train"])
            n = min(len(tl), len(cap["train"]))
            print("  envelope", kind, e2, "max rel train-loss dev",
                  float(np.max(np.abs(tl[:n] - cap["train"][:n]) / np.array(cap["train"][:n]))),
                  "mae", m2[1]["mae"], "vs", metrics[1]["mae"])
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"), seed=np.int64(seed),
            lat_checksums=np.array([checksum(l) for l in lat]),
            label_checksums=np.array([checksum(l) for l in labels]),
            train_losses=np.array(cap["train"]), valid_losses=np.array(cap["valid"]),
            **{"final_" + k.replace(".", "_"): v.numpy() for k, v in cap["model"].items()})
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump({"args": args, "noise": noise, "flip_valid": flip, "before": metrics[0],
                       "after": metrics[1], "events": events, "files": files,
                       "text_files": text, "envelope": env}, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
