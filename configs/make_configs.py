"""Hyper-parameter grid of the reference's random search (configs/make_configs.py:16-61).

    python configs/make_configs.py [--seed S] [--out DIR]

Writes DIR/config_<i>.json for every point of the 512-point grid below and
DIR/../<name>.csv (one row per config, with its config_num), like the
reference.  The reference shuffles with the unseeded global `random`, so its
config_<i>.json differs from run to run; `--seed` makes the numbering
reproducible (default: unseeded, the reference's behaviour).  The committed
multimodal_search/config_0.json and multimodal_search.csv come from --seed 0.
"""
import argparse
import csv
import itertools
import json
import os
import random

PARAMS = {  # make_configs.py:16-31, same keys and value order
    "sentiment_hidden_size": [100, 150],
    "lr": [1e-3, 1e-4],
    "sentiment_lr": [1e-1, 1e-2],
    "seq_len": [20],
    "word_sim_metric": ["angular"],
    "n_epochs": [100, 200],
    "freeze_weights": [False],
    "n_sentiment_epochs": [400],
    "word_loss_weight": [0.001, 0.002],
    "likelihood_weight": [0.0001, 0.001],
    "pos_embed_dim": [2, 4],
    "e2e": [True],
    "norm": ["layer_norm", "batch_norm"],
    "optimizer": ["sgd", "adam"],
}


def grid():
    keys = list(PARAMS)
    return [dict(zip(keys, vals)) for vals in itertools.product(*PARAMS.values())]


def main(argv=None):
    here = os.path.dirname(os.path.realpath(__file__))
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--name", default="multimodal_search")
    ap.add_argument("--out", default=None, help="output folder (default: configs/<name>)")
    a = ap.parse_args(argv)
    folder = a.out or os.path.join(here, a.name)
    os.makedirs(folder, exist_ok=True)
    configs = grid()
    print(len(configs))
    (random.Random(a.seed) if a.seed is not None else random).shuffle(configs)
    with open(os.path.join(os.path.dirname(folder), f"{a.name}.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(PARAMS) + ["config_num"])
        w.writeheader()
        for i, c in enumerate(configs):
            c["config_num"] = i
            with open(os.path.join(folder, f"config_{i}.json"), "w") as g:
                json.dump(c, g)
            w.writerow(c)
    return configs


if __name__ == "__main__":
    main()
