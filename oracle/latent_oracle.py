"""CPU restatement of the latent-optimisation likelihoods — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import
this module, as the checker; the product path (libmmb + the mirror) never
does.  Pinned against tests/golden/g7_*, g8_matrix (made by running the
reference's own functions, tests/golden/make_goldens_latent.py).

torch on the CPU in float32, the reference's own arithmetic order:
  normal_log_prob       losses.py:13-33
  word_log_prob_angular2 losses.py:68-95 (cosine via x/|x| . y/|y| with the
                        1e-8 norm clamp of torch.nn.CosineSimilarity)
  log_prob_matrix       losses.py:216-274
"""
from __future__ import annotations

import math

import torch

COS_EPS = 1e-8


def _cos(x, y):
    """torch cosine_similarity(x, y, dim=-1): each side divided by its clamped
    norm, then the product summed."""
    xn = torch.linalg.vector_norm(x, dim=-1, keepdim=True).clamp_min(COS_EPS)
    yn = torch.linalg.vector_norm(y, dim=-1, keepdim=True).clamp_min(COS_EPS)
    return ((x / xn) * (y / yn)).sum(-1)


def normal_log_prob(mu, sigma, values, mask):
    """losses.py:13-33 (mu, sigma [B,1,F]; values, mask [B,T,F])."""
    var = sigma * sigma
    lp = torch.log(1. / torch.sqrt(2. * math.pi * var)) - (values - mu) ** 2 / (2. * var)
    return (lp * mask).squeeze().sum(-1).sum(-1)


def word_log_prob_angular2(latents, table, word_weights, sent, mask, a):
    """losses.py:68-95: lp [B]."""
    c_all = _cos(latents[:, None, :], table[None, :, :])           # [B, V]
    Z = (1. - torch.acos(c_all) / math.pi).sum(-1, keepdim=True)  # [B, 1]
    alpha = 1. / (Z * a + 1.)
    score = 1. - torch.acos(_cos(sent, latents[:, None, :])) / math.pi
    lp = torch.log(alpha * word_weights + (1. - alpha) * score / Z)
    return (lp * mask[:, :, 0]).sum(-1)


def log_prob_matrix(args, latents, out, data, masks, word_fn):
    """losses.py:216-274 (without the inf exit)."""
    word = word_fn(latents, data["text_weights"], data["text"], masks["text"])
    lps = {k: normal_log_prob(d["mu"][:, None], d["sigma"][:, None], data[k], masks[k])
           for k, d in out.items()}
    if "word_loss_weight" in args:
        ww = args["word_loss_weight"]
        return sum(lps.values()) * ((1. - ww) / len(lps)) + ww * word
    return sum(lps.values()) + word
