"""Drop-in for `/root/reference/sentiment_model.py` — the sentiment regressor (a10-a12).

Same classes and functions, same arguments, same printed/saved artefacts.
The arithmetic runs on the GPU through libmmb:

* SentimentModel.forward          -> mmb_mlp_forward (no-grad calls); while autograd
  records (the e2e joint objective, simplesif.py:776-790) -> the autograd
  Function _Regressor: mmb_mlp_forward_train / mmb_mlp_backward
* predict_sentiment / validation  -> mmb_mlp_eval (per-batch L1 means + predictions)
* train_sentiment inner loop      -> mmb_mlp_train: every mini-batch step of a
  block of epochs (forward, L1 backward, SGD) in ONE single-workgroup launch,
  parameters updated in place in the model's own tensors.

Mini-batch order is the reference's: the DataLoaders are still shuffled by the
global torch RNG, and we consume it exactly as iterating them would
(`_epoch_batches`), so with the same seed the same rows meet the same weights.
Host<->device syncs happen once per validation (every `valid_niter` epochs),
where the reference's early-stopping logic needs the loss on the host.

Deviation kept small and documented: loss histories are returned as Python
floats (the reference returns 0-d tensors).
"""
from __future__ import annotations

import os
import json

import numpy as np
import torch
import torch.nn as nn
import torch.optim as optim
from torch.utils.data import DataLoader, Dataset

import mmb_lib as L
from losses import full_loss, iemocap_loss, pom_loss


class SentimentData(Dataset):
    """sentiment_model.py:14-27."""

    def __init__(self, sentiment, device):
        super(Dataset, self).__init__()
        if not torch.is_tensor(sentiment):
            sentiment = torch.tensor(sentiment, device=device, dtype=torch.float32)
        self.sentiment = sentiment

    def __len__(self):
        return self.sentiment.size()[0]

    def __getitem__(self, idx):
        return idx, self.sentiment[idx]


def _dims(model):
    h, d = model.hidden1.weight.shape
    o = model.out.weight.shape[0]
    return d, h, o


def _params(model):
    ps = (model.hidden1.weight, model.hidden1.bias, model.out.weight, model.out.bias)
    for p in ps:
        if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
            raise L.MMBError("SentimentModel parameters must be contiguous float32 on the GPU "
                             "(call .to(device) with a cuda device)")
    return ps


class _Regressor(torch.autograd.Function):
    """y = relu(x W1^T + b1) W2^T + b2 with a hand-written backward
    (libmmb mmb_mlp_forward_train / mmb_mlp_backward): gradients to the
    inputs (the latents, in the e2e loop) and to every parameter."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        x = x.detach().contiguous()
        b, d = x.shape
        h, o = w1.shape[0], w2.shape[0]
        y = torch.empty((b, o), dtype=torch.float32, device=x.device)
        hid = torch.empty((b, h), dtype=torch.float32, device=x.device)
        L.call("mmb_mlp_forward_train", L.ptr(x), b, d, h, o, L.ptr(w1.detach()),
               L.ptr(b1.detach()), L.ptr(w2.detach()), L.ptr(b2.detach()), L.ptr(y), L.ptr(hid),
               L.stream_ptr())
        ctx.save_for_backward(x, hid, w1, w2)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, hid, w1, w2 = ctx.saved_tensors
        b, d = x.shape
        h, o = w1.shape[0], w2.shape[0]
        need = ctx.needs_input_grad
        e = lambda *shape: torch.empty(shape, dtype=torch.float32, device=x.device)
        dx = e(b, d) if need[0] else None
        dw1, db1 = (e(h, d) if need[1] else None), (e(h) if need[2] else None)
        dw2, db2 = (e(o, h) if need[3] else None), (e(o) if need[4] else None)
        dh = e(b, h)
        L.call("mmb_mlp_backward", L.ptr(x), L.ptr(hid), b, d, h, o, L.ptr(w1.detach()),
               L.ptr(w2.detach()), L.ptr(dy.float().contiguous()), L.ptr(dh), L.ptr(dx),
               L.ptr(dw1), L.ptr(db1), L.ptr(dw2), L.ptr(db2), L.stream_ptr())
        return dx, dw1, db1, dw2, db2


class SentimentModel(nn.Module):
    """sentiment_model.py:29-41: squeeze(out(relu(hidden1(x))))."""

    def __init__(self, embedding_dim, hidden_dim, n_out):
        super(SentimentModel, self).__init__()
        self.hidden1 = nn.Linear(embedding_dim, hidden_dim)
        self.out = nn.Linear(hidden_dim, n_out)

    def forward(self, inputs):
        dev = self.hidden1.weight.device
        if dev.type != "cuda":
            raise L.MMBError("SentimentModel runs on the GPU (libmmb); move it with .to('cuda')")
        if torch.is_grad_enabled() and (inputs.requires_grad or
                                        any(p.requires_grad for p in self.parameters())):
            # differentiable forward (the e2e joint objective, simplesif.py:776-790)
            w1, b1, w2, b2 = _params(self)
            x = inputs.to(dev, torch.float32)
            lead = x.shape[:-1]
            y = _Regressor.apply(x.reshape(-1, x.shape[-1]), w1, b1, w2, b2)
            return y.reshape(*lead, w2.shape[0]).squeeze()
        home = inputs.device
        x = inputs.detach().to(dev, torch.float32)
        lead = x.shape[:-1]
        x = x.reshape(-1, x.shape[-1]).contiguous()
        d, h, o = _dims(self)
        w1, b1, w2, b2 = _params(self)
        y = torch.empty((x.shape[0], o), dtype=torch.float32, device=dev)
        with torch.no_grad():
            L.call("mmb_mlp_forward", L.ptr(x), None, x.shape[0], d, h, o, L.ptr(w1), L.ptr(b1),
                   L.ptr(w2), L.ptr(b2), L.ptr(y), L.stream_ptr())
        return y.reshape(*lead, o).squeeze().to(home)


def save_sentiment(path, model):
    torch.save(model.state_dict(), os.path.join(path, "senti.bin"))


def load_sentiment(path, embedding_dim, hidden_dim, device, n_out=1):
    """sentiment_model.py:46-50 (the reference omits n_out and cannot run; default 1 here)."""
    model = SentimentModel(embedding_dim, hidden_dim, n_out)
    model.load_state_dict(torch.load(path, weights_only=True))
    return model.to(device)


def _epoch_batches(loader):
    """Index batches of one pass over `loader`, consuming the global torch RNG
    exactly as `for j, senti in loader` does (the iterator's base seed, then
    the RandomSampler's seed), without collating any rows."""
    it = iter(loader)  # draws _base_seed (dataloader.py _BaseDataLoaderIter.__init__)
    batches = [torch.as_tensor(b, dtype=torch.int64) for b in loader.batch_sampler]
    del it
    return batches


def _epoch_perm(loader):
    """The sample order of one pass over `loader`, consuming the global torch
    RNG exactly as `for j, senti in loader` does -- for the reference's
    loaders (shuffle=True, default RandomSampler, no generator): the
    iterator's base seed, then the sampler's seed and its randperm
    (dataloader.py _BaseDataLoaderIter.__init__, sampler.py
    RandomSampler.__iter__), one int64 tensor instead of 40 batch lists.
    Anything else takes _epoch_batches."""
    from torch.utils.data import BatchSampler, RandomSampler

    s = loader.sampler
    n = len(loader.dataset)
    if (type(s) is RandomSampler and s.generator is None and not s.replacement
            and loader.generator is None and s.num_samples == n
            and type(loader.batch_sampler) is BatchSampler and not loader.drop_last):
        torch.empty((), dtype=torch.int64).random_()  # the iterator's _base_seed
        seed = int(torch.empty((), dtype=torch.int64).random_().item())
        g = torch.Generator()
        g.manual_seed(seed)
        return torch.randperm(n, generator=g)
    batches = _epoch_batches(loader)
    return torch.cat(batches) if batches else torch.zeros(0, dtype=torch.int64)


def _labels(loader, dev):
    y = loader.dataset.sentiment.to(dev, torch.float32)
    return y.reshape(y.shape[0], -1).contiguous()


def _f32_mean_of(values, count):
    """epoch_loss += loss.mean() ... / n  in float32, as the reference's tensors do."""
    s = np.float32(0.0)
    for v in values:
        s = np.float32(s + np.float32(v))
    return float(np.float32(s / np.float32(count)))


def _evaluate(loader, model, latents, dev):
    """One shuffled pass: per-batch mean L1, predictions in loader order."""
    d, h, o = _dims(model)
    w1, b1, w2, b2 = _params(model)
    batches = _epoch_batches(loader)
    n = sum(len(b) for b in batches)
    perm = torch.cat(batches).to(dev) if batches else torch.zeros(0, dtype=torch.int64, device=dev)
    lab = _labels(loader, dev)
    lat = latents.detach().to(dev, torch.float32).contiguous()
    nb = len(batches)
    bl = torch.empty(max(nb, 1), dtype=torch.float32, device=dev)
    pred = torch.empty((max(n, 1), o), dtype=torch.float32, device=dev)
    L.call("mmb_mlp_eval", L.ptr(lat), L.ptr(lab), L.ptr(perm), n, loader.batch_size, d, h, o,
           L.ptr(w1), L.ptr(b1), L.ptr(w2), L.ptr(b2), L.ptr(bl), L.ptr(pred), L.stream_ptr())
    return bl[:nb], pred[:n], perm, lab


def predict_sentiment(data, model, latents):
    """sentiment_model.py:52-74 — returns (predictions, y_test) as numpy in loader order."""
    dev = model.hidden1.weight.device
    n_samples = len(data.dataset)
    _, pred, perm, lab = _evaluate(data, model, latents, dev)
    y = lab[perm]
    total_loss = (pred - y).abs().sum()
    print("MAE: {}".format(total_loss / n_samples))
    if pred.shape[1] == 1:
        pred, y = pred[:, 0], y[:, 0]
    return pred.cpu().numpy(), y.cpu().numpy()


def train_sentiment(args, model, train_data, train_latents, valid_data, valid_latents,
                    model_loader, valid_niter=10, verbose=False, model_save_path=None):
    """sentiment_model.py:76-163: SGD on mean L1 over shuffled batches of 32,
    validation every `valid_niter` epochs, optional early stopping with
    patience 10 / 3 trials / lr decay and best-model reload.

    The epochs AND the validation passes run inside mmb_mlp_train: without
    early stopping the whole run is one launch and one read-back; with it,
    one launch per stretch of epochs ending at a validation (the host's
    early-stopping decision -- checkpoint, reload, lr decay, stop -- needs
    that validation loss before the next epoch).  The sample orders are drawn
    from the global torch RNG in the reference's order (each epoch's training
    pass, then the validation pass where i % valid_niter == 0)."""
    n_epochs = args["n_sentiment_epochs"]
    lr = args["sentiment_lr"]
    patience = 10
    n_trials = 3
    dev = model.hidden1.weight.device
    d, h, o = _dims(model)
    w1, b1, w2, b2 = _params(model)
    n_samples = len(train_data.dataset)
    optimizer = optim.SGD(model.parameters(), lr=lr)  # state_dict-compatible checkpoints
    lat = train_latents.detach().to(dev, torch.float32).contiguous()
    lab = _labels(train_data, dev)
    B = train_data.batch_size
    spe = (n_samples + B - 1) // B
    n_valid = len(valid_data.dataset)
    vlat = valid_latents.detach().to(dev, torch.float32).contiguous()
    vlab = _labels(valid_data, dev)
    in_kernel = valid_data.batch_size == B and n_valid > 0
    nbv = (n_valid + B - 1) // B if in_kernel else 0
    ws = torch.zeros(L.query("mmb_mlp_workspace_bytes", d, h) // 4 + 4, dtype=torch.float32,
                     device=dev)  # zeroed once: the launch leaves its control words zero
    flag = torch.zeros(1, dtype=torch.int32, device=dev)

    def run(i, block, lr):
        """Epochs i .. i + block - 1: per-step losses [block, spe] and the
        per-batch losses of each validation in the stretch (host arrays)."""
        perms, vperms = [], []
        for e in range(i, i + block):
            perms.append(_epoch_perm(train_data))
            if in_kernel and e % valid_niter == 0:
                vperms.append(_epoch_perm(valid_data))
        perm = torch.cat(perms).to(dev)
        step_loss = torch.empty(spe * block, dtype=torch.float32, device=dev)
        if in_kernel and vperms:
            vperm = torch.cat(vperms).to(dev)
            vloss = torch.empty(len(vperms) * nbv, dtype=torch.float32, device=dev)
            vargs = (L.ptr(vlat), L.ptr(vlab), L.ptr(vperm), n_valid, valid_niter, i, L.ptr(vloss))
        else:
            vloss = None
            vargs = (None, None, None, 0, 1, i, None)
        L.call("mmb_mlp_train", L.ptr(lat), L.ptr(lab), L.ptr(perm), n_samples, block, B, d, h, o,
               float(lr), L.ptr(w1), L.ptr(b1), L.ptr(w2), L.ptr(b2), L.ptr(step_loss), *vargs,
               L.ptr(ws), L.ptr(flag), L.stream_ptr())
        out = torch.cat([step_loss, vloss]) if vloss is not None else step_loss
        host = out.cpu().numpy()  # the one read-back of the stretch
        if int(flag.item()) & L.MMB_FLAG_SYNC_TIMEOUT:
            raise RuntimeError("mmb_mlp_train: the exchange between its workgroups timed out; "
                               "the regressor's parameters are invalid")
        sl = host[:spe * block].reshape(block, spe)
        vl = host[spe * block:].reshape(len(vperms), nbv) if vloss is not None else None
        return sl, vl

    train_losses, valid_losses = [], []
    n_bad = 0
    n_bad_trials = 0
    i = 0
    last_epoch_loss = 0.0
    while i < n_epochs:
        if args["early_stopping"]:  # stop at the next validation: the host decides there
            block = 1 if i % valid_niter == 0 else min(valid_niter - i % valid_niter + 1,
                                                       n_epochs - i)
        else:
            block = n_epochs - i
        if not in_kernel:
            block = 1 if i % valid_niter == 0 else min(valid_niter - i % valid_niter, n_epochs - i)
        sl, vl = run(i, block, lr)
        stop = False
        k = 0
        for e in range(block):
            ep = i + e
            train_losses.append(_f32_mean_of(sl[e], spe))
            last_epoch_loss = float(np.float32(np.sum(sl[e], dtype=np.float32)))
            if ep % valid_niter != 0:
                continue
            if in_kernel:
                avg_valid_loss = _f32_mean_of(vl[k], nbv)
            else:
                bl, _, _, _ = _evaluate(valid_data, model, valid_latents, dev)
                bl = bl.cpu().numpy()
                avg_valid_loss = _f32_mean_of(bl, len(bl))
            k += 1
            print("Epoch {}: {} (avg val loss {})".format(ep, train_losses[-1], avg_valid_loss))
            is_better = len(valid_losses) == 0 or avg_valid_loss < min(valid_losses)
            valid_losses.append(avg_valid_loss)
            if args["early_stopping"]:
                if is_better:
                    n_bad = 0
                    if model_save_path is not None:
                        torch.save({"model_state_dict": model.state_dict(),
                                    "optimizer_state_dict": optimizer.state_dict()},
                                   os.path.join(model_save_path, "senti.bin"))
                else:
                    print("patience {}".format(n_bad))
                    n_bad += 1
                    if n_bad >= patience:
                        n_bad_trials += 1
                        if n_bad_trials < n_trials:
                            if model_save_path is not None:
                                print("reloading model and decaying learning rate...")
                                ck = torch.load(os.path.join(model_save_path, "senti.bin"),
                                                weights_only=True)
                                model.load_state_dict(ck["model_state_dict"])
                                optimizer.load_state_dict(ck["optimizer_state_dict"])
                            lr = lr * args["lr_decay"]
                            for g in optimizer.param_groups:
                                g["lr"] = lr
                            n_bad = 0
                        else:
                            print("early stopping...")
                            stop = True
        i += block
        if stop:
            break
    print("Epoch {}: {}".format(i - 1, last_epoch_loss / n_samples))
    return train_losses, valid_losses


def train_sentiment_for_latents(args, latents, sentiment_data, device, verbose=False,
                                model_save_path=None, train_idxes=None):
    """sentiment_model.py:165-265 (including its quirk: after early stopping
    the best model is reloaded into a new module that is then not used)."""
    dev = L.require_gpu() if torch.device(device).type != "cuda" else torch.device(device)
    train_latents, valid_latents, test_latents = latents
    hidden_dim = args["sentiment_hidden_size"]
    embedding_dim = train_latents.size()[-1]
    train, valid, test = sentiment_data
    n_out = 1 if train.ndim == 1 else train.shape[-1]
    senti_model = SentimentModel(embedding_dim, hidden_dim, n_out).to(dev)
    print("train data shape:", train.shape)
    print("train latents shape:", train_latents.size())
    if train_idxes is not None:
        train = train[train_idxes]
        train_latents = train_latents[train_idxes]
        print("train data shape:", train.shape)
        print("train latents shape:", train_latents.size())
    train_data = SentimentData(train, dev)
    valid_data = SentimentData(valid, dev)
    test_data = SentimentData(test, dev)
    assert train_latents.size()[0] == train.shape[0]
    print("# of sentiment points:", len(train_data))
    train_loader = DataLoader(train_data, batch_size=32, shuffle=True)
    valid_loader = DataLoader(valid_data, batch_size=32, shuffle=True)
    test_loader = DataLoader(test_data, batch_size=32, shuffle=True)

    metric = {"mosi": full_loss, "iemocap": iemocap_loss}.get(args["dataset"], pom_loss)

    print("Initial sentiment predictions")
    senti_model.eval()
    predictions, y_test = predict_sentiment(test_loader, senti_model, test_latents)
    results = metric(predictions, y_test)
    if model_save_path is not None:
        if "accuracy" in results:
            with open(os.path.join(model_save_path, "test_acc_before.txt"), "w") as f:
                f.write(str(results["accuracy"]))
        with open(os.path.join(model_save_path, "test_results_before.json"), "w") as f:
            json.dump(results, f, indent=2)

    print("Training sentiment model on sentence embeddings...")
    senti_model.train()
    model_loader = lambda: load_sentiment(model_save_path, embedding_dim, hidden_dim, dev, n_out)
    train_losses, valid_losses = train_sentiment(args, senti_model, train_loader, train_latents,
                                                 valid_loader, valid_latents, model_loader,
                                                 verbose=verbose, model_save_path=model_save_path)
    if model_save_path is not None:
        with open(os.path.join(model_save_path, "senti_train_loss.txt"), "w") as f:
            for loss in train_losses:
                f.write("{}\n".format(loss))
        with open(os.path.join(model_save_path, "senti_valid_loss.txt"), "w") as f:
            for loss in valid_losses:
                f.write("{}\n".format(loss))
    if not args["early_stopping"]:
        if model_save_path is not None:
            save_sentiment(model_save_path, senti_model)
    else:
        print("reloading best")
        model = SentimentModel(embedding_dim, hidden_dim, n_out).to(dev)
        checkpoint = torch.load(os.path.join(model_save_path, "senti.bin"), weights_only=True)
        model.load_state_dict(checkpoint["model_state_dict"])

    print("Sentiment predictions after training")
    senti_model.eval()
    predictions, y_test = predict_sentiment(test_loader, senti_model, test_latents)
    results = metric(predictions, y_test)
    if model_save_path is not None:
        if "accuracy" in results:
            with open(os.path.join(model_save_path, "test_acc_after.txt"), "w") as f:
                f.write(str(results["accuracy"]))
        with open(os.path.join(model_save_path, "test_results_after.json"), "w") as f:
            json.dump(results, f, indent=2)
    print("-----------------------------")
    return results
