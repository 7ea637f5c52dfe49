"""CPU restatement of the sentiment regressor loop (a10/a11) — TEST INFRASTRUCTURE ONLY.

Follows `/root/reference/sentiment_model.py`:
  SentimentModel            :29-41   squeeze(out(relu(hidden1(x))))
  predict_sentiment         :52-74   one shuffled pass, L1 sums
  train_sentiment           :76-163  SGD on mean L1 over shuffled batches of 32,
                                      validation every 10 epochs, early stopping
                                      (patience 10, 3 trials, lr decay, best reload)
  train_sentiment_for_latents :165-265 init, test predictions before/after,
                                      the reload-best quirk (:243-250: a NEW model
                                      is built -- consuming the torch RNG -- and
                                      then not used)

torch on the CPU, consuming the global torch RNG in the reference's order (model
init, then each DataLoader pass draws its iterator base seed and its sampler
permutation), so with the same `torch.manual_seed` the same rows meet the same
weights.  The best-model checkpoint is kept in memory (a torch.save / torch.load
round trip of a state dict is exact).  Used by the CPU tests (against the
reference fixtures g5_*) and as bench.py's regressor cpu_baseline.
"""
from __future__ import annotations

import copy

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.data import DataLoader, Dataset


class _Labels(Dataset):
    def __init__(self, y):
        self.y = torch.as_tensor(y, dtype=torch.float32)

    def __len__(self):
        return self.y.shape[0]

    def __getitem__(self, i):
        return i, self.y[i]


class Regressor(nn.Module):
    def __init__(self, d, h, o):
        super().__init__()
        self.hidden1 = nn.Linear(d, h)
        self.out = nn.Linear(h, o)

    def forward(self, x):
        return self.out(F.relu(self.hidden1(x))).squeeze()


def predict(loader, model, lat):
    preds, ys = [], []
    with torch.no_grad():
        for j, y in loader:
            preds.append(model(lat[j]))
            ys.append(y)
    return torch.cat(preds).numpy(), torch.cat(ys).numpy()


def train(args, model, train_loader, train_lat, valid_loader, valid_lat, valid_niter=10):
    """sentiment_model.py:76-163; returns (train_losses, valid_losses, events)."""
    lr = args["sentiment_lr"]
    patience, n_trials = 10, 3
    opt = torch.optim.SGD(model.parameters(), lr=lr)
    train_losses, valid_losses = [], []
    n_bad = n_bad_trials = 0
    best = None
    events = {"reloads": 0, "early_stop": False}
    for i in range(args["n_sentiment_epochs"]):
        epoch_loss = torch.zeros(())
        nb = 0
        for j, y in train_loader:
            nb += 1
            model.zero_grad()
            loss = (model(train_lat[j]) - y).abs()
            epoch_loss = epoch_loss + loss.mean()
            loss.mean().backward()
            opt.step()
        train_losses.append(float(epoch_loss / nb))
        if i % valid_niter == 0:
            vl = torch.zeros(())
            vb = 0
            with torch.no_grad():
                for j, y in valid_loader:
                    vl = vl + (model(valid_lat[j]) - y).abs().mean()
                    vb += 1
            v = float(vl / vb)
            is_better = len(valid_losses) == 0 or v < min(valid_losses)
            valid_losses.append(v)
            if args["early_stopping"]:
                if is_better:
                    n_bad = 0
                    best = (copy.deepcopy(model.state_dict()), copy.deepcopy(opt.state_dict()))
                else:
                    n_bad += 1
                    if n_bad >= patience:
                        n_bad_trials += 1
                        if n_bad_trials < n_trials:
                            model.load_state_dict(best[0])
                            opt.load_state_dict(best[1])
                            events["reloads"] += 1
                            lr = lr * args["lr_decay"]
                            for g in opt.param_groups:
                                g["lr"] = lr
                            n_bad = 0
                        else:
                            events["early_stop"] = True
                            break
    return train_losses, valid_losses, events


def train_for_latents(args, latents, labels, batch=32):
    """sentiment_model.py:165-265 with metrics left to the caller: returns
    dict(before=(pred, y), after=(pred, y), train_losses, valid_losses,
    state, events).  Call `torch.manual_seed(s)` first, like the reference run."""
    tr, va, te = (torch.as_tensor(l, dtype=torch.float32) for l in latents)
    ytr, yva, yte = labels
    n_out = 1 if ytr.ndim == 1 else ytr.shape[-1]
    model = Regressor(tr.shape[-1], args["sentiment_hidden_size"], n_out)
    loaders = [DataLoader(_Labels(y), batch_size=batch, shuffle=True) for y in (ytr, yva, yte)]
    model.eval()
    before = predict(loaders[2], model, te)
    model.train()
    tl, vl, events = train(args, model, loaders[0], tr, loaders[1], va)
    if args["early_stopping"]:
        Regressor(tr.shape[-1], args["sentiment_hidden_size"], n_out)  # :244, RNG only
    model.eval()
    after = predict(loaders[2], model, te)
    return {"before": before, "after": after, "train_losses": tl, "valid_losses": vl,
            "state": {k: v.detach().clone() for k, v in model.state_dict().items()},
            "events": events}
