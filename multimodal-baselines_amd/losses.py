"""Drop-in for `/root/reference/losses.py`.

* Latent-optimisation likelihoods (losses.py:13-274):
  same names and signatures, computed by libmmb kernels with hand-written
  backward passes (`latent.py`, csrc/latent_kernels.hip): the angular word
  model without the [B, V, 300] broadcast, the Gaussians from masked frame
  sums.  The dot-product word model (losses.py:98-151) is not on any
  configured path (make_configs.py:21-22 only uses 'angular'; the CLI even
  calls it with one argument too many, simplesif.py:509,528) and stays plain
  torch on the device.
* Evaluation metrics (losses.py:276-366) run on the host (numpy +
  scikit-learn) exactly as in the reference: O(N) bookkeeping on a few
  hundred predictions.  Quirks kept: the weighted F1
  passes (y_pred, y_true) swapped (losses.py:291), POM values are rounded lists.
"""
from __future__ import annotations

import sys

import numpy as np
import torch
from sklearn.metrics import (accuracy_score, classification_report, confusion_matrix,
                             f1_score)

import latent as LT


# ------------------------------------------------------------------ likelihoods
def _sum_last2_of_squeezed(lp_rows, shape):
    """`masked_log_prob.squeeze().sum(-1).sum(-1)` (losses.py:33) from per-row
    sums: the squeeze drops unit axes of [B, T, F], so fewer than three
    non-unit axes collapse the batch too (B = 1 or T = 1 give one scalar)."""
    if sum(1 for s in shape if s != 1) >= 3:
        return lp_rows
    return lp_rows.sum()


def get_normal_log_prob(mu, sigma, values, mask):
    """losses.py:13-33: mu, sigma [B, 1, F]; values, mask [B, T, F]."""
    B, T, F = values.shape
    stats = LT.GaussStats(text=LT.gauss_stats(values, mask))
    mu2 = mu.reshape(B, F)
    sg2 = sigma.reshape(B, F)
    lp = LT.gauss_log_prob(stats, ["text"], [mu2], [sg2])[0]
    return _sum_last2_of_squeezed(lp, (B, T, F))


def get_word_log_prob_angular(latents, weights, word_embeddings, data, mask, a):
    """losses.py:36-66: token ids `data` [B, L]; weights [V]; mask [B, L]."""
    table = LT.word_table(word_embeddings)
    ids = data.to(latents.device)
    w = weights.to(latents.device)[ids.long()]
    m = torch.as_tensor(mask, device=latents.device, dtype=torch.float32).expand(ids.shape)
    return LT.word_log_prob(latents, table, w, m, a, ids=ids)


def get_word_log_prob_angular2(latents, word_embeddings, word_weights, sent_embeddings, mask, a):
    """losses.py:68-95: sentence rows sent_embeddings [B, L, D], word_weights
    [B, L], mask [B, L, D] (its first feature column is used, :92)."""
    table = LT.word_table(word_embeddings)
    m = mask[:, :, 0]
    return LT.word_log_prob(latents, table, word_weights, m, a, sent_dense=sent_embeddings)


def get_word_log_prob_dot_prod(latents, weights, word_embeddings, data, a):
    """losses.py:98-124 (Arora's softmax model; not on a configured path)."""
    Z_s = latents.matmul(word_embeddings.transpose(0, 1)).exp().sum(-1, keepdim=True)
    alpha = 1. / (Z_s * a + 1.)
    dot = torch.bmm(word_embeddings[data], latents.unsqueeze(-1)).squeeze()
    return torch.log(alpha * weights[data] + (1. - alpha) * dot.exp() / Z_s).sum(dim=-1)


def get_word_log_prob_dot_prod2(latents, word_embeddings, word_weights, sent_embeddings, mask, a):
    """losses.py:126-151."""
    Z_s = latents.matmul(word_embeddings.transpose(0, 1)).exp().sum(-1, keepdim=True)
    alpha = 1. / (Z_s * a + 1.)
    dot = torch.bmm(sent_embeddings, latents.unsqueeze(-1)).squeeze()
    lp = torch.log(alpha * word_weights + (1. - alpha) * dot.exp() / Z_s)
    return (lp * mask[:, :, 0]).sum(dim=-1)


def _combine(args, log_probs: dict, word_log_prob):
    """losses.py:258-274: the inf check (exits like the reference) and the weighting."""
    if log_probs:
        mins = torch.stack([lp.detach().min() for lp in log_probs.values()]).abs().cpu()
        bad = False
        for (m, _), v in zip(log_probs.items(), mins):
            if float(v) == np.inf:
                print(m, "inf")
                bad = True
        if bad:
            sys.exit()
    if "word_loss_weight" in args:
        word_weight = args["word_loss_weight"]
        other_weight = (1. - word_weight) / len(log_probs)
        return sum(log_probs.values()) * other_weight + word_weight * word_log_prob
    return sum(log_probs.values()) + word_log_prob


def combine_weighted(args, log_probs: dict, word_log_prob):
    """_combine's weighting without its host-side inf check (the caller
    checks, e.g. once per captured step: simplesif.check_step)."""
    if "word_loss_weight" in args:
        word_weight = args["word_loss_weight"]
        other_weight = (1. - word_weight) / len(log_probs)
        return sum(log_probs.values()) * other_weight + word_weight * word_log_prob
    return sum(log_probs.values()) + word_log_prob


def get_log_prob_matrix(args, latents, out, data, masks, word_log_prob_fn,
                        device=torch.device("cpu"), verbose=False):
    """losses.py:216-274: word model + one Gaussian per generator output key."""
    word_log_prob = word_log_prob_fn(latents, data["text_weights"], data["text"], masks["text"])
    log_probs = {}
    for modality, d in out.items():
        log_probs[modality] = get_normal_log_prob(d["mu"].unsqueeze(1), d["sigma"].unsqueeze(1),
                                                  data[modality], masks[modality])
    return _combine(args, log_probs, word_log_prob)


def get_log_prob_matrix_old(args, latents, audio, visual, data, masks, word_log_prob_fn,
                            device=torch.device("cpu"), verbose=False):
    """losses.py:153-214 (audio/visual-only generator)."""
    word_log_prob = word_log_prob_fn(latents, data["text"], masks["text"])
    lps = {"audio": get_normal_log_prob(audio[0].unsqueeze(1), audio[1].unsqueeze(1),
                                        data["covarep"], masks["covarep"]),
           "visual": get_normal_log_prob(visual[0].unsqueeze(1), visual[1].unsqueeze(1),
                                         data["facet"], masks["facet"])}
    bad = False
    for k, lp in lps.items():
        if float(lp.min().abs()) == np.inf:
            print({"audio": "aud", "visual": "vis"}[k] + " inf")
            bad = True
    if bad:
        sys.exit()
    if verbose:
        print("Visual: {}\tAudio: {}\tWord: {}".format(lps["visual"].min(), lps["audio"].min(),
                                                       word_log_prob.min()))
    if "word_loss_weight" in args:
        ww = args["word_loss_weight"]
        o = (1. - ww) / 2
        return o * lps["audio"] + o * lps["visual"] + ww * word_log_prob
    return lps["audio"] + lps["visual"] + word_log_prob


def full_loss(predictions, y_test, verbose=True):
    """MOSI metrics (losses.py:276-315)."""
    predictions = np.asarray(predictions).flatten()
    y_test = np.asarray(y_test).flatten()
    mae = np.mean(np.absolute(predictions - y_test))
    corr = np.corrcoef(predictions, y_test)[0][1]
    mult = round(sum(np.round(predictions) == np.round(y_test)) / float(len(y_test)), 5)
    f_score = round(f1_score(np.round(predictions), np.round(y_test), average="weighted"), 5)
    true_label = (y_test >= 0)
    predicted_label = (predictions >= 0)
    accuracy = accuracy_score(true_label, predicted_label)
    confusion_mat = confusion_matrix(true_label, predicted_label)
    class_report = classification_report(true_label, predicted_label, digits=5, output_dict=True)
    if verbose:
        print("mae: {}".format(mae))
        print("corr: {}".format(corr))
        print("mult_acc: {}".format(mult))
        print("mult f_score: {}".format(f_score))
        print("Confusion Matrix :")
        print(confusion_mat)
        print("Classification Report :")
        print(classification_report(true_label, predicted_label, digits=5))
        print("Accuracy {}".format(accuracy))
    return {
        "mae": float(mae),
        "accuracy": float(accuracy),
        "corr": float(corr),
        "mult_acc": float(mult),
        "f_score": float(f_score),
        "confusion_matrix": confusion_mat.tolist(),
        "class_report": class_report,
    }


def iemocap_loss(predictions, y_test, verbose=True):
    """IEMOCAP metrics (losses.py:317-340)."""
    all_true_label = np.argmax(y_test, axis=1)
    all_predicted_label = np.argmax(predictions, axis=1)
    f_score = f1_score(all_true_label, all_predicted_label, average="weighted")
    accuracy = accuracy_score(all_true_label, all_predicted_label)
    confusion_mat = confusion_matrix(all_true_label, all_predicted_label)
    class_report = classification_report(all_true_label, all_predicted_label, digits=5,
                                         output_dict=True)
    if verbose:
        print("F1 score:", f_score)
        print("Accuracy:", accuracy)
        print("Confusion Matrix :")
        print(confusion_mat)
        print("Classification Report :")
        print(classification_report(all_true_label, all_predicted_label, digits=5))
    return {
        "accuracy": float(accuracy),
        "f_score": float(f_score),
        "confusion_matrix": confusion_mat.tolist(),
        "class_report": class_report,
    }


def pom_loss(predictions, y_test, verbose=True):
    """POM metrics, one value per label column (losses.py:342-366)."""
    predictions = np.asarray(predictions)
    y_test = np.asarray(y_test)
    mae = np.mean(np.absolute(predictions - y_test), axis=0)
    mae = [round(a, 3) for a in mae]
    corr = [round(np.corrcoef(predictions[:, i], y_test[:, i])[0][1], 3)
            for i in range(y_test.shape[1])]
    mult = [round(sum(np.round(predictions[:, i]) == np.round(y_test[:, i])) / float(len(y_test)), 3)
            for i in range(y_test.shape[1])]
    f_score = [round(f1_score(np.round(predictions[:, i]), np.round(y_test[:, i]),
                              average="weighted"), 5) for i in range(y_test.shape[1])]
    if verbose:
        print("mae:", mae)
        print("corr:", corr)
        print("mult_acc:", mult)
        print("f_score:", f_score)
    return {
        "mae": [float(x) for x in mae],
        "corr": [float(x) for x in corr],
        "mult_acc": [float(x) for x in mult],
        "f_score": [float(x) for x in f_score],
    }
