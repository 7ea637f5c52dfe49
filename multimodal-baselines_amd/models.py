"""Parameter layout of the MMB generators (consumed by the closed-form MMB2 path).

Mirrors the *parameter layout* of `models.AudioVisualGeneratorMultimodal`
(`/root/reference/models.py:107-202`): a ModuleDict keyed by modality
combination, each holding ``{'mu', 'log_sigma'}: nn.Linear(D, F_k)``.  The
closed-form estimate (`sif2.py:164-208`) reads only ``.weight [F_k, D]`` and
``.bias [F_k]`` of those layers.  Construction order matches the reference so
``torch.manual_seed(s)`` reproduces the reference's initial weights bit for bit.

The generator *forward* (latent-optimisation objective)
runs all twelve linears as ONE GEMM over their concatenated weights (the
reference's per-key `nn.Linear` calls, `/root/reference/models.py:187-202`,
are the same dot products; only the GEMM grouping differs): one forward GEMM
and two backward GEMMs instead of 36 small ones, one `exp` for all the
sigmas, and the per-key mu / sigma outputs are column views of the result
(the Gaussian kernels take row strides, `mmb_gauss_loglik_strided`).  The
parameters, their layout and their initialisation stay per key.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import latent as LT

# fixed key order of sif2.py:167-174 (also the ModuleDict order, models.py:134-159)
MMB2_KEYS = ("audio", "visual", "audiovisual", "textaudio", "textvisual", "textaudiovisual")
MMB1_KEYS = ("audio", "visual")


def combo_dims(key: str, D: int, A: int, Vd: int) -> list[tuple[str, int]]:
    """Segments (modality, width) that make up combination ``key``'s features.

    Order is the torch.cat order used by the callers (simplesif.py:825-830):
    text first, then audio, then visual.
    """
    segs = []
    if key.startswith("text"):
        segs.append(("text", D))
    if "audio" in key:
        segs.append(("audio", A))
    if "visual" in key:
        segs.append(("visual", Vd))
    return segs


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm (same parameters, state-dict keys and forward) whose
    backward on the device is one libmmb launch (`latent.layer_norm`, f32
    only); CPU tensors (the host-side tests) and other dtypes (a generator cast
    to .double() / .half()) take torch's, as nn.LayerNorm would."""

    def forward(self, x):
        if (x.is_cuda and self.weight is not None and self.bias is not None
                and x.dtype == self.weight.dtype == self.bias.dtype == torch.float32
                and self.weight.is_cuda):
            return LT.layer_norm(x, self.weight, self.bias, self.eps)
        return super().forward(x)


class AudioVisualGeneratorMultimodal(nn.Module):
    def __init__(self, embedding_dim, audio_dim, visual_dim, norm=None, frozen_weights=True,
                 unimodal=False):
        super().__init__()
        self.embedding = None
        self.embedding_dim = embedding_dim
        keys = MMB1_KEYS if unimodal else MMB2_KEYS
        layers = {}
        for k in keys:
            width = sum(w for _, w in combo_dims(k, embedding_dim, audio_dim, visual_dim))
            layers[k] = nn.ModuleDict({
                "mu": nn.Linear(embedding_dim, width),
                "log_sigma": nn.Linear(embedding_dim, width),
            })
        self.embed2out = nn.ModuleDict(layers)
        if norm is None:
            self.norm = None
        elif norm == "layer_norm":
            self.norm = LayerNorm(embedding_dim)
        elif norm == "batch_norm":
            self.norm = nn.BatchNorm1d(embedding_dim)
        else:
            raise NotImplementedError
        if frozen_weights:
            self.freeze_weights()

    def freeze_weights(self):
        for p in self.embed2out.parameters():
            p.requires_grad = False

    def init_embedding(self, embedding):
        assert embedding.size()[-1] == self.embedding_dim
        self.embedding = embedding
        self.embedding.requires_grad = True
        self.embedding_dim = self.embedding.size()[-1]

    def forward(self, embeddings):
        """{key: {'mu': x W_mu^T + b_mu, 'sigma': exp(x W_ls^T + b_ls)}} with x
        the (normalised) embeddings (models.py:187-202): y = x [W_mu; W_ls]^T
        + [b_mu; b_ls] in one GEMM, every key's block a column view of y."""
        x = self.norm(embeddings) if self.norm is not None else embeddings
        mods = list(self.embed2out.values())
        w = torch.cat([m["mu"].weight for m in mods] + [m["log_sigma"].weight for m in mods])
        b = torch.cat([m["mu"].bias for m in mods] + [m["log_sigma"].bias for m in mods])
        widths = [m["mu"].out_features for m in mods]
        f = sum(widths)
        mu, ls = F.linear(x, w, b).split([f, f], dim=-1)
        mus = mu.split(widths, dim=-1)
        sigmas = ls.exp().split(widths, dim=-1)
        return {k: {"mu": mus[i], "sigma": sigmas[i]} for i, k in enumerate(self.embed2out)}

    def networks(self):
        """``{key: (mu_linear, log_sigma_linear)}`` as built at simplesif.py:853-856."""
        return {k: (m["mu"], m["log_sigma"]) for k, m in self.embed2out.items()}
