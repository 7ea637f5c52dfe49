"""Drop-in for `/root/reference/simplesif.py` — the CLI.

    python simplesif.py CONFIG {mosi,pom,iemocap} [--unimodal] [--pos_embed_dim N]
        [--batch_size 64] [--n_runs 1] [--semi_sup_idxes 0.1..0.9] [--config_name NAME]
        [--lr_decay 0.5] [--early_stopping] [--sentiment_epochs N]
        [--emotion {happy,angry,neutral,sad}] [--optimizer {sgd,adam}]
        [--norm {layer_norm,batch_norm}] [--likelihood_weight W] [--e2e {y,n}]
        [--time_test] [--cuda_device {0..3}] [--cuda]

Same arguments, same config JSON (configs/make_configs.py), same run tree
(model_saves/<config_name>/config_<n>_run_<r>/{config.json, pre/embed.bin,
post/embed.bin, embed_*loss.txt, post/senti*.txt|bin, post/test_*}), same
printed milestones.  The work runs on the MI355X whether or not --cuda is
given (libmmb has no CPU path):

  SIF sentence embeddings (per split)      sif.get_sentence_embeddings   (HIP a1-a5)
  word + Gaussian likelihoods, backward    latent.py                     (HIP, §8f row 1)
  closed-form MMB2 (--time_test)           sif2.estimate_embedding_overall_gpu2 (HIP a6-a8)
  regressor training / evaluation          sentiment_model               (HIP a10-a12)

The training loops, optimisers (torch.optim SGD / Adam), generator modules and
DataLoader shuffling are the reference's, so a run consumes the torch RNG in
the same order and a seeded run tracks the reference run.  What changes is the
objective's evaluation: per split, the masked frame sums of every modality are
streamed once (`latent.GaussStats`), and a batch's log-likelihood is computed
from those sums and the batch's token ids (`Objective.log_prob`), with the
reference's values — nothing [B, T, F] or [B, V, 300] is built per step.
"""
from __future__ import annotations

import argparse
import json
import os
import pprint
import sys
import time

import numpy as np
import torch
import torch.nn as nn
import torch.optim as optim
from torch.utils.data import DataLoader

import latent as LT
import mmb_lib as L
from losses import _combine, combine_weighted
from models import AudioVisualGeneratorMultimodal
from sentiment_model import SentimentData, SentimentModel, train_sentiment_for_latents
from sif import get_sentence_embeddings, load_weights
from sif2 import estimate_embedding_overall_gpu2
from utils import MMData, MMDataExtra, add_positional_embeddings, load_data, normalize_data

WORD_A = 1e-3  # simplesif.py:513


def update_masks(mask_dict, data, embedding_dim):
    """simplesif.py:36-40: text mask = (ids != 0) broadcast over the embedding."""
    tmp = (data != 0).astype(int)
    mask_dict["text"] = np.broadcast_to(np.expand_dims(tmp, -1), tmp.shape + (embedding_dim,))
    print(np.all(mask_dict["text"][:, :, 1] == mask_dict["text"][:, :, 0]))


def update_masks_vect(mask_dict, data, key="text"):
    """simplesif.py:42-47: 1 where every feature of the frame is non-zero."""
    tmp2 = np.all(data != 0, axis=-1).astype(int)
    print(tmp2.shape)
    mask_dict[key] = np.broadcast_to(np.expand_dims(tmp2, -1), data.shape)


def read_config(config_file):
    with open(config_file, "r") as f:
        config = json.load(f)
    pprint.PrettyPrinter(indent=2).pprint(config)
    return config


def parse_arguments(argv=None):
    """simplesif.py:186-238 (including: --likelihood_weight is parsed but the
    config's value is used; e2e 'y'/'n' strings become booleans)."""
    p = argparse.ArgumentParser()
    p.add_argument("config_file", help="JSON file containing hyperparameters for model")
    p.add_argument("dataset", choices=["mosi", "pom", "iemocap"])
    p.add_argument("--unimodal", action="store_true", help="run mmb1 (unimodal factorization)")
    p.add_argument("--pos_embed_dim", type=int)
    p.add_argument("--batch_size", type=int, default=64)
    p.add_argument("--n_runs", type=int, default=1)
    p.add_argument("--semi_sup_idxes", choices=["{:.1f}".format(x) for x in np.arange(0.1, 1, 0.1)])
    p.add_argument("--config_name", help="override config name in config file")
    p.add_argument("--lr_decay", type=float, default=0.5)
    p.add_argument("--early_stopping", action="store_true",
                   help="early stopping when training sentiment model")
    p.add_argument("--sentiment_epochs", type=int)
    p.add_argument("--emotion", choices=["happy", "angry", "neutral", "sad"], help="iemocap emotion")
    p.add_argument("--optimizer", choices=["sgd", "adam"], default="sgd")
    p.add_argument("--norm", choices=["layer_norm", "batch_norm"])
    p.add_argument("--likelihood_weight", type=float)
    p.add_argument("--e2e", choices=["y", "n"], help="end-to-end training of latent variables")
    p.add_argument("--time_test", action="store_true", help="Run inference timing")
    p.add_argument("--cuda_device", type=int, choices=list(range(4)), help="set CUDA device number")
    p.add_argument("--cuda", action="store_true")
    args = vars(p.parse_args(argv))
    override = {}
    if args["pos_embed_dim"] is not None:
        override["pos_embed_dim"] = args["pos_embed_dim"]
    if args["e2e"] is not None:
        override["e2e"] = args["e2e"]
    config = read_config(args["config_file"])
    print("######################################")
    print("Config: {}".format(config["config_num"]))
    args.update(config)
    args.update(override)
    if args["e2e"] == "y":
        args["e2e"] = True
    elif args["e2e"] == "n":
        args["e2e"] = False
    if args["sentiment_epochs"]:
        args["n_sentiment_epochs"] = args["sentiment_epochs"]
    return args


# ------------------------------------------------------------------ objective
class Objective:
    """The latent objective of one data split (losses.get_log_prob_matrix as
    the CLI calls it, simplesif.py:93-131,735-773), precomputed for the split:
    token ids / weights / mask of the word model and the masked frame sums of
    the text (aligned), audio and visual streams."""

    def __init__(self, args, table: "LT.WordTable", weights32, ids, gauss_text, gauss_text_mask,
                 audio, audio_mask, visual, visual_mask):
        dev = table.table.device
        self.args, self.table = args, table
        self.ids = torch.as_tensor(np.asarray(ids), device=dev).to(torch.int32).contiguous()
        self.w = weights32[self.ids.long()].contiguous()
        self.m = (self.ids != 0).to(torch.float32).contiguous()
        self.stats = LT.GaussStats(
            text=LT.gauss_stats(torch.as_tensor(gauss_text, device=dev, dtype=torch.float32),
                                torch.as_tensor(gauss_text_mask, device=dev, dtype=torch.float32)),
            audio=LT.gauss_stats(torch.as_tensor(audio, device=dev, dtype=torch.float32),
                                 torch.as_tensor(audio_mask, device=dev, dtype=torch.float32)),
            visual=LT.gauss_stats(torch.as_tensor(visual, device=dev, dtype=torch.float32),
                                  torch.as_tensor(visual_mask, device=dev, dtype=torch.float32)))

    def parts(self, latents, out, j):
        """(word log-prob [B], Gaussian log-probs [K, B], keys) for batch rows j
        (device work only: no host sync, so it can be captured in a graph)."""
        j = j.to(self.ids.device)
        word = LT.word_log_prob(latents, self.table, self.w[j], self.m[j], WORD_A, ids=self.ids[j])
        keys = list(out.keys())
        lp = LT.gauss_log_prob(self.stats, keys, [out[k]["mu"] for k in keys],
                               [out[k]["sigma"] for k in keys], idx=j)
        return word, lp, keys

    def log_prob(self, latents, out, j):
        """get_log_prob_matrix(...) [B] for batch rows j of the split."""
        word, lp, keys = self.parts(latents, out, j)
        wmin = word.detach().min().abs()
        if float(wmin) == np.inf:  # simplesif.py:517-523
            print("word inf")
            print(latents.size())
            sys.exit()
        return _combine(self.args, {k: lp[i] for i, k in enumerate(keys)}, word)

    def log_prob_nocheck(self, latents, out, j):
        """log_prob without the host-side inf checks, plus the values those
        checks read: (log-prob [B], [word min |.|, per-key min |.| ...])."""
        word, lp, keys = self.parts(latents, out, j)
        mins = torch.cat([word.detach().min().abs().view(1), lp.detach().amin(dim=1).abs()])
        return combine_weighted(self.args, {k: lp[i] for i, k in enumerate(keys)}, word), mins


def sigma_mins(out):
    """|min sigma| for the per-step 'boo!' check, as device values: one min
    over the generator's whole sigma block when the keys' sigmas are column
    views of one tensor (models.py's fused head), else one per key.  check_step
    reads which form it got from its length."""
    sigs = [d["sigma"] for d in out.values()]
    base = sigs[0]._base
    if base is not None and all(t._base is base for t in sigs) and base.dim() == 2 and \
            sum(t.shape[1] for t in sigs) == base.shape[1]:
        return base.detach().amin().abs().view(1)
    return torch.stack([t.detach().min() for t in sigs]).abs()


def check_step(out, mins_all, latents_size, n_sig=None):
    """The reference's per-step host checks, in its order, from one device
    read: sigma < 1e-7 prints (simplesif.py:82-84 / 724-726), a word
    log-prob of inf exits (simplesif.py:517-523), a Gaussian one of inf
    exits (losses.py:258-264).  mins_all = [loss, sigma mins (n_sig: K, or 1
    from sigma_mins' whole-block form), word min, Gaussian mins (K)]; returns
    the loss.  With one block minimum the per-key minima are read from `out`
    only when it is below the threshold (the step's tensors are still intact:
    the next replay has not been launched)."""
    v = mins_all.cpu().numpy()
    K = len(out)
    ns = K if n_sig is None else n_sig
    if ns == K:
        per_key = v[1:1 + K]
    elif float(v[1]) < 1e-7:
        per_key = torch.stack([d["sigma"].detach().min() for d in out.values()]).abs().cpu().numpy()
    else:
        per_key = [1.0] * K
    for (modality, d), m in zip(out.items(), per_key):
        if float(m) < 1e-7:
            print(d, "boo!")
    if float(v[1 + ns]) == np.inf:
        print("word inf")
        print(latents_size)
        sys.exit()
    bad = False
    for k, m in zip(out.keys(), v[2 + ns:]):
        if float(m) == np.inf:
            print(k, "inf")
            bad = True
    if bad:
        sys.exit()
    return float(v[0])


USE_GRAPHS = os.environ.get("MMB_STEP_GRAPHS", "1") != "0"


class StepGraphs:
    """One optimisation step's device work -- generator forward, objective,
    regressor, backward -- captured as a HIP graph per batch size and
    replayed, so the ~100 small launches of a step cost one graph launch.

    `body(j)` (j: a device index tensor) must do device work only and return
    (out dict, tensor of the values the host checks read).  The optimiser step
    stays eager (torch.optim, the reference's arithmetic), as do the host
    checks, which read the step's values once per step like the reference's
    float() calls.  Gradients: a replay overwrites the gradient buffers its
    capture allocated (what zero_grad + backward produce); after a replay the
    parameters' .grad are pointed at that graph's buffers.  Capture needs
    warm-up passes; module buffers (BatchNorm running statistics) are
    restored after them, so the first real step sees the same state as the
    reference's.

    Host / device overlap (r03): the batch's indices go up from a pinned
    buffer without blocking, and the checked values come back into a pinned
    buffer behind an event, so a caller can launch the optimiser step BEFORE
    it waits for them (`step()`): the optimiser's kernels run while the host
    reads the values and runs the checks.  Only the order of the host-side
    effects moves -- a check that exits does so with the step's optimiser
    update already applied to parameters the process then discards; the
    printed `out` tensors are the step's own (the next replay has not been
    launched)."""

    def __init__(self, body, modules, params, device):
        self.body, self.modules, self.params, self.dev = body, modules, list(params), device
        self.graphs = {}

    def _capture(self, b):
        dev = self.dev
        j = torch.zeros(b, dtype=torch.int64, device=dev)
        bufs = [x for m in self.modules for x in m.buffers()]
        saved = [x.clone() for x in bufs]
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(2):
                for p in self.params:
                    p.grad = None
                self.body(j)
        torch.cuda.current_stream(dev).wait_stream(side)
        with torch.no_grad():
            for x, v in zip(bufs, saved):
                x.copy_(v)
        for p in self.params:
            p.grad = None
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            outs = self.body(j)
        j_pin = torch.empty(b, dtype=torch.int64).pin_memory()
        vals_pin = torch.empty(outs[1].shape, dtype=outs[1].dtype).pin_memory()
        self.graphs[b] = (g, j, outs, [p.grad for p in self.params], j_pin, vals_pin,
                          torch.cuda.Event())

    def launch(self, j_host):
        """Replay the step for index batch `j_host`; returns (out, vals) with
        vals a pinned host tensor that is valid after `wait()`."""
        b = len(j_host)
        if b not in self.graphs:
            self._capture(b)
        g, j, outs, grads, j_pin, vals_pin, ev = self.graphs[b]
        j_pin.copy_(j_host)  # (the previous step's wait() has retired its upload)
        j.copy_(j_pin, non_blocking=True)
        g.replay()
        vals_pin.copy_(outs[1], non_blocking=True)
        ev.record()
        for p, gr in zip(self.params, grads):
            p.grad = gr
        self._ev = ev
        return outs[0], vals_pin

    def wait(self):
        self._ev.synchronize()

    def step(self, j_host, optimizer):
        """launch + optimizer.step() + wait: the optimiser's kernels are queued
        before the host blocks on the values."""
        out, vals = self.launch(j_host)
        optimizer.step()
        self.wait()
        return out, vals

    def __call__(self, j_host):
        out, vals = self.launch(j_host)
        self.wait()
        return out, vals


def _sigma_check(out):
    """simplesif.py:82-84 ('boo!' print), one device sync for all keys."""
    mins = torch.stack([d["sigma"].detach().min() for d in out.values()]).abs().cpu()
    for (modality, d), v in zip(out.items(), mins):
        if float(v) < 1e-7:
            print(d, "boo!")


def optimize_latents(args, train: bool, gen_model, embed_arr, dataloader, n_epochs, lr, objective,
                     device, validation_data=None, verbose=True):
    """simplesif.py:49-162."""
    embeddings = torch.tensor(np.array(embed_arr, copy=True), device=device, dtype=torch.float32)
    embeddings.requires_grad = True
    grad_params = [embeddings]
    if train and not args["freeze_weights"]:
        grad_params.extend(gen_model.parameters())
    if args["optimizer"] == "sgd":
        optimizer = optim.SGD(grad_params, lr=lr)
    elif args["optimizer"] == "adam":
        optimizer = optim.Adam(grad_params, lr=lr)
    valid_niter = 10
    start_time = time.time()
    losses = []
    all_valid_losses = []
    graphs = None
    if USE_GRAPHS:
        def body(j):
            e = embeddings[j]  # one gather for both uses (see the e2e body below)
            out = gen_model(e)
            sig = sigma_mins(out)
            lp, mins = objective.log_prob_nocheck(e, out, j)
            avg_log_prob = (-lp).mean()
            avg_log_prob.backward()
            return out, torch.cat([avg_log_prob.detach().view(1), sig, mins])

        graphs = StepGraphs(body, [gen_model], grad_params, device)
    for i in range(n_epochs):
        epoch_loss = 0.
        iters = 0
        for j in _index_batches(dataloader):
            iters += 1
            if graphs is not None:
                out, vals = graphs.step(j, optimizer)
                epoch_loss += check_step(out, vals, embeddings[:len(j)].size(),
                                         len(vals) - 2 - len(out))
                continue
            optimizer.zero_grad()
            out = gen_model(embeddings[j])
            _sigma_check(out)
            log_prob = -objective.log_prob(embeddings[j], out, j)
            avg_log_prob = log_prob.mean()
            avg_log_prob.backward()
            optimizer.step()
            epoch_loss += float(avg_log_prob)
        losses.append(epoch_loss)
        if i % valid_niter == 0:
            if verbose:
                print("epoch {}: {} ({}s)".format(i, epoch_loss / iters, time.time() - start_time))
            if validation_data is not None and i % (valid_niter * 8) == 0:
                valid_embedding, valid_loader, valid_obj = validation_data
                _, valid_losses = optimize_latents(args, False, gen_model, valid_embedding,
                                                   valid_loader, n_epochs, lr, valid_obj, device,
                                                   verbose=False)
                print("Validation loss:", valid_losses[-1])
                all_valid_losses.append(valid_losses[-1])
    if validation_data is not None:
        valid_embedding, valid_loader, valid_obj = validation_data
        _, valid_losses = optimize_latents(args, False, gen_model, valid_embedding, valid_loader,
                                           n_epochs, lr, valid_obj, device, verbose=False)
        print("(Final) Validation loss:", valid_losses[-1])
        all_valid_losses.append(valid_losses[-1])
    embeddings.requires_grad = False
    return embeddings, (losses, all_valid_losses)


def _index_batches(loader):
    """The index batches `for x in loader` yields as x[0], consuming the torch
    RNG exactly as iterating the reference's MMData loader does: the iterator
    draws its base seed on creation, a RandomSampler its own seed on the first
    batch; no rows are collated."""
    it = iter(loader)
    del it
    for b in loader.batch_sampler:
        yield torch.as_tensor(b, dtype=torch.int64)


# ------------------------------------------------------------------ main
def main(argv=None):
    args = parse_arguments(argv)
    if args["cuda_device"]:  # simplesif.py:243 (0 is ignored: truthiness)
        os.environ["CUDA_VISIBLE_DEVICES"] = str(args["cuda_device"])
    device = L.require_gpu()

    word2ix, word_embeddings, data = load_data(args)
    train, valid, test = data
    train, train_mask = normalize_data(train)
    valid, valid_mask = normalize_data(valid)
    test, test_mask = normalize_data(test)
    text_key = "text" if args["dataset"] == "mosi" else "text_id"
    for d, m in ((train, train_mask), (valid, valid_mask), (test, test_mask)):
        update_masks(m, d[text_key], word_embeddings.shape[-1])
    n_train = train["label"].shape[0]

    weights = load_weights(args)
    if args["word_sim_metric"] == "dot_prod":
        word_embeddings = word_embeddings / np.linalg.norm(word_embeddings, axis=-1, keepdims=True)

    train_embedding = get_sentence_embeddings(word_embeddings, weights, train[text_key])
    valid_embedding = get_sentence_embeddings(word_embeddings, weights, valid[text_key])
    test_embedding = get_sentence_embeddings(word_embeddings, weights, test[text_key])
    combined_embedding = np.concatenate([train_embedding, valid_embedding, test_embedding], axis=0)

    weights = torch.tensor(weights, device=device, dtype=torch.float32)
    word_embeddings = torch.tensor(word_embeddings, device=device, dtype=torch.float32)
    for d, m in ((train, train_mask), (valid, valid_mask), (test, test_mask)):
        ids_t = torch.as_tensor(d[text_key], device=device).long()
        if args["dataset"] == "mosi":
            d["text_id"] = d["text"]
        else:
            d["text_align"] = d["text"]
            update_masks_vect(m, d["text_align"], "text_align")
        d["text"] = word_embeddings[ids_t]
        d["text_weights"] = weights[ids_t]

    print("# pos embeddings:", args["pos_embed_dim"])
    if "pos_embed_dim" in args and args["pos_embed_dim"] > 0:
        for d, m in ((train, train_mask), (valid, valid_mask), (test, test_mask)):
            d["covarep"] = add_positional_embeddings(args, d["covarep"])
            d["facet"] = add_positional_embeddings(args, d["facet"])
            n_points, seq_len = m["covarep"].shape[:2]
            ext = np.ones((n_points, seq_len, args["pos_embed_dim"]), dtype=np.int64)
            m["covarep"] = np.concatenate([m["covarep"], ext], axis=-1)
            m["facet"] = np.concatenate([m["facet"], ext], axis=-1)
    else:
        print("not adding positional embeddings!")

    BATCH_SIZE = args["batch_size"]
    table = LT.word_table(word_embeddings)

    def split_objective(d, m):
        # the Gaussian text stream and its per-frame mask (broadcast over the
        # features, as update_masks / update_masks_vect build it)
        if args["dataset"] == "mosi":
            gt, gm = d["text"], (np.asarray(d["text_id"]) != 0)
        else:
            gt, gm = d["text_align"], np.all(np.asarray(d["text_align"]) != 0, axis=-1)
        gm = torch.as_tensor(gm.astype(np.float32), device=device)[:, :, None]
        return Objective(args, table, weights, d["text_id"], gt, gm,
                         d["covarep"], m["covarep"], d["facet"], m["facet"])

    def dataset(d, m):
        if args["dataset"] == "mosi":
            return MMData(d["text"], d["covarep"], d["facet"], m, d["text_weights"], device)
        return MMDataExtra(d["text"], d["covarep"], d["facet"], m, d["text_weights"],
                           d["text_align"], device)

    train_obj, valid_obj, test_obj = (split_objective(train, train_mask),
                                      split_objective(valid, valid_mask),
                                      split_objective(test, test_mask))
    train_dataset = dataset(train, train_mask)
    valid_dataset = dataset(valid, valid_mask)
    test_dataset = dataset(test, test_mask)
    dataloader = DataLoader(train_dataset, batch_size=BATCH_SIZE, shuffle=True)
    valid_dataloader = DataLoader(valid_dataset, batch_size=BATCH_SIZE * 8)
    test_dataloader = DataLoader(test_dataset, batch_size=BATCH_SIZE * 8)
    print("# batches: {}".format(len(train_dataset) // BATCH_SIZE))

    EMBEDDING_DIM = train["text"].shape[-1]
    AUDIO_DIM = train["covarep"].shape[-1]
    VISUAL_DIM = train["facet"].shape[-1]
    print(EMBEDDING_DIM)

    sentiment_data = (train["label"], valid["label"], test["label"])
    sentiment_train_idxes = None
    senti_mask = (torch.zeros(n_train, device=device) if args["dataset"] == "mosi"
                  else torch.zeros(n_train, 1, device=device))
    if args["semi_sup_idxes"] is not None:
        import h5py  # the reference's subset file (simplesif.py:496-501)

        with h5py.File("{}_subset_idxes.h5".format(args["dataset"]), "r") as f:
            sentiment_train_idxes = f[args["semi_sup_idxes"]][:]
            print("semi-supervised sentiment idxes:", sentiment_train_idxes.shape)
            senti_mask[sentiment_train_idxes] = 1.
    print(senti_mask.size())

    if args["word_sim_metric"] not in ("angular", "dot_prod"):
        raise NotImplementedError
    if args["word_sim_metric"] == "dot_prod":
        # simplesif.py:509,528 hands the 5-argument get_word_log_prob_dot_prod
        # six arguments: the reference fails on its first batch
        raise TypeError("get_word_log_prob_dot_prod() takes 5 positional arguments but 6 were given")

    config_name = args["config_name"] or os.path.split(os.path.split(args["config_file"])[0])[1]

    def run_folder(r):
        folder = "model_saves/{}/config_{}_run_{}".format(config_name, args["config_num"], r)
        os.makedirs(folder, exist_ok=True)
        with open(os.path.join(folder, "config.json"), "w") as f:
            json.dump(args, f, indent=2)
        pre_path, post_path = os.path.join(folder, "pre"), os.path.join(folder, "post")
        os.makedirs(pre_path, exist_ok=True)
        os.makedirs(post_path, exist_ok=True)
        torch.save(torch.tensor(combined_embedding.copy(), device=device, dtype=torch.float32),
                   os.path.join(pre_path, "embed.bin"))
        return folder, post_path

    def write_lines(path, values):
        with open(path, "w") as f:
            for v in values:
                f.write("{}\n".format(v))

    def new_generator():
        return AudioVisualGeneratorMultimodal(EMBEDDING_DIM, AUDIO_DIM, VISUAL_DIM, norm=args["norm"],
                                              frozen_weights=args["freeze_weights"],
                                              unimodal=args["unimodal"]).to(device)

    if not args["e2e"]:
        for i in range(args["n_runs"]):
            folder, post_path = run_folder(i)
            gen_model = new_generator()
            print("Training one at a time...")
            lr = args["lr"]
            N_EPOCHS = args["n_epochs"]
            train_embed, (train_losses, valid_losses) = optimize_latents(
                args, True, gen_model, train_embedding, dataloader, N_EPOCHS, lr, train_obj, device,
                validation_data=(valid_embedding, valid_dataloader, valid_obj))
            write_lines(os.path.join(folder, "embed_loss.txt"), train_losses)
            write_lines(os.path.join(folder, "embed_valid_loss.txt"), valid_losses)
            valid_embed, _ = optimize_latents(args, False, gen_model, valid_embedding,
                                              valid_dataloader, N_EPOCHS, lr, valid_obj, device)
            test_embed, test_losses = optimize_latents(args, False, gen_model, test_embedding,
                                                       test_dataloader, N_EPOCHS, lr, test_obj,
                                                       device)
            write_lines(os.path.join(folder, "embed_test_loss.txt"), test_losses)
            torch.save(torch.cat([train_embed, valid_embed, test_embed], dim=0),
                       os.path.join(post_path, "embed.bin"))
            print("$$$$$$$$$$$$$$$$$$$$$$$$$$$$$$$$$")
            print("Initial sentiment predictions, AFTER optimizing audio and visual")
            train_sentiment_for_latents(args, (train_embed, valid_embed, test_embed), sentiment_data,
                                        device, train_idxes=sentiment_train_idxes,
                                        model_save_path=post_path)
        sys.stdout.flush()
        return

    print("end-to-end training of latents")
    train_s, valid_s, test_s = sentiment_data
    senti_train_data = SentimentData(train_s, device)
    for r in range(args["n_runs"]):
        folder, post_path = run_folder(r)
        gen_model = new_generator()
        n_out = 1 if train["label"].ndim == 1 else train["label"].shape[-1]
        senti_model = SentimentModel(EMBEDDING_DIM, args["sentiment_hidden_size"], n_out).to(device)
        train_embed = torch.tensor(train_embedding.copy(), device=device, dtype=torch.float32)
        train_embed.requires_grad = True
        grad_params = [train_embed]
        grad_params.extend(gen_model.parameters())
        grad_params.extend(senti_model.parameters())
        lr = args["lr"]
        if args["optimizer"] == "sgd":
            optimizer = optim.SGD(grad_params, lr=lr)
        elif args["optimizer"] == "adam":
            optimizer = optim.Adam(grad_params, lr=lr)
        loss_function = nn.L1Loss(reduction="none")
        start_time = time.time()
        valid_niter = 10
        train_losses = []
        all_valid_losses = []
        N_EPOCHS = args["n_epochs"]
        graphs = None
        if USE_GRAPHS:
            senti_labels = senti_train_data.sentiment
            lw = args["likelihood_weight"]

            def body(j):
                # ONE gather of the batch's latents for the generator, the
                # objective and the regressor (the reference indexes three
                # times: three sort-based index backwards and two dense adds
                # of the [N, 300] gradient per step; here the three gradient
                # contributions are summed on the [B, 300] rows and scattered
                # once -- the same three terms per row)
                e = train_embed[j]
                out = gen_model(e)
                sig = sigma_mins(out)
                lp, mins = train_obj.log_prob_nocheck(e, out, j)
                senti_loss = loss_function(senti_model(e), senti_labels[j])
                if sentiment_train_idxes is not None:
                    senti_loss = senti_loss * senti_mask[j]
                senti_loss = senti_loss.mean(dim=-1)
                loss = lw * (-lp) + (1 - lw) * senti_loss
                lm = loss.mean()
                lm.backward()
                return out, torch.cat([lm.detach().view(1), sig, mins])

            graphs = StepGraphs(body, [gen_model, senti_model], grad_params, device)
        for i in range(N_EPOCHS):
            epoch_loss = 0.
            iters = 0
            for j in _index_batches(dataloader):
                if graphs is not None:
                    iters += 1
                    out, vals = graphs.step(j, optimizer)
                    epoch_loss += check_step(out, vals, train_embed[:len(j)].size(),
                                             len(vals) - 2 - len(out))
                    continue
                _, s_data = senti_train_data[j]
                iters += 1
                optimizer.zero_grad()
                out = gen_model(train_embed[j])
                _sigma_check(out)
                log_prob = -train_obj.log_prob(train_embed[j], out, j)
                senti_predict = senti_model(train_embed[j])
                senti_loss = loss_function(senti_predict, s_data)
                if sentiment_train_idxes is not None:
                    senti_loss *= senti_mask[j.to(device)]
                senti_loss = senti_loss.mean(dim=-1)
                loss = args["likelihood_weight"] * log_prob + (1 - args["likelihood_weight"]) * senti_loss
                loss.mean().backward()
                epoch_loss += float(loss.mean())
                optimizer.step()
            train_losses.append(epoch_loss)
            if i % valid_niter == 0:
                print("epoch {}: {} ({}s)".format(i, epoch_loss / iters, time.time() - start_time))
                if i % (valid_niter * 8) == 0:
                    _, (valid_losses, _) = optimize_latents(args, False, gen_model, valid_embedding,
                                                            valid_dataloader, N_EPOCHS, lr,
                                                            valid_obj, device, verbose=False)
                    print("Validation loss:", valid_losses[-1])
                    all_valid_losses.append(valid_losses[-1])

        valid_embed, _ = optimize_latents(args, False, gen_model, valid_embedding, valid_dataloader,
                                          N_EPOCHS, lr, valid_obj, device)
        test_embed, (test_losses, _) = optimize_latents(args, False, gen_model, test_embedding,
                                                        test_dataloader, N_EPOCHS, lr, test_obj,
                                                        device)
        if args["time_test"]:
            time_test(args, gen_model, test, test_mask, word_embeddings, weights, device)
            print(train_embed.size())
            print(valid_embed.size())
            print(test_embed.size())
            sys.exit()

        write_lines(os.path.join(folder, "embed_loss.txt"), train_losses)
        write_lines(os.path.join(folder, "embed_valid_loss.txt"), all_valid_losses)
        write_lines(os.path.join(folder, "embed_test_loss.txt"), test_losses)
        torch.save(torch.cat([train_embed, valid_embed, test_embed], dim=0),
                   os.path.join(post_path, "embed.bin"))
        print("$$$$$$$$$$$$$$$$$$$$$$$$$$$$$$$$$")
        print("Initial sentiment predictions, AFTER optimizing audio and visual")
        train_embed.requires_grad = False
        valid_embed.requires_grad = False
        test_embed.requires_grad = False
        train_sentiment_for_latents(args, (train_embed, valid_embed, test_embed), sentiment_data,
                                    device, train_idxes=sentiment_train_idxes,
                                    model_save_path=post_path)
        sys.stdout.flush()
    sys.stdout.flush()


def time_test(args, gen_model, test, test_mask, word_embeddings, weights, device):
    """simplesif.py:808-880: closed-form MMB2 embeddings of the test split, timed.
    (The reference concatenates the unaligned text with the aligned frames,
    :821-830, which only lines up for MOSI.)"""
    text = torch.as_tensor(test["text"], dtype=torch.float, device=device)
    audio = torch.as_tensor(test["covarep"], dtype=torch.float, device=device)
    visual = torch.as_tensor(test["facet"], dtype=torch.float, device=device)
    test_data = {"text": text, "audio": audio, "visual": visual,
                 "audiovisual": torch.cat([audio, visual], dim=-1),
                 "textaudio": torch.cat([text, audio], dim=-1),
                 "textvisual": torch.cat([text, visual], dim=-1),
                 "textaudiovisual": torch.cat([text, audio, visual], dim=-1)}
    keys = ["audio", "visual", "audiovisual", "textaudio", "textvisual", "textaudiovisual"]
    test_masks = {k: None for k in keys}  # indexed by key, never read (sif2.py:182)
    networks = {k: (gen_model.embed2out[k]["mu"], gen_model.embed2out[k]["log_sigma"]) for k in keys}
    text_tmp = torch.as_tensor(test["text_id"], dtype=torch.long, device=device)
    sentence_weights = torch.where(text_tmp >= 0, weights[text_tmp.clamp(min=0)],
                                   torch.zeros((), device=device))
    embeddings = word_embeddings[text_tmp, :]
    torch.cuda.synchronize()
    start_time = time.time()
    with torch.no_grad():
        latents = estimate_embedding_overall_gpu2(test_data, test_masks, networks,
                                                  sentence_weights, embeddings)
    torch.cuda.synchronize()
    end_time = time.time()
    print("time taken:", end_time - start_time)
    print("#############################################")
    print(test.keys())
    print(test_mask.keys())
    return latents


if __name__ == "__main__":
    main()
