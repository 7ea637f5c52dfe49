"""Drop-in for the live part of `/root/reference/sif2.py` — closed-form MMB2.

* calc_weights(data, b_mean, b_log_sigma, mask)                 sif2.py:103-114
* estimate_embedding_overall_gpu2(data, masks, networks,
                                  sentence_weights, embeddings) sif2.py:164-208

Same arguments and result ([N, 300] fp32, unit rows, no PC removal).  Instead
of materialising q_mean/q_sigma [N,T,F_k] for six combinations and running
twelve matmuls, one streaming kernel reduces every utterance's frames to the
per-feature sums of x and x^2, and one fp32-MFMA GEMM against the merged
generator matrix finishes the embedding (see csrc/mm2_kernels.hip for the
algebra).  The concatenated combination tensors in `data` are not read: by
construction (simplesif.py:825-830) they are torch.cat of data['text'],
data['audio'] and data['visual'], which are what the kernel streams.  The
reference ignores `masks` too (pads contribute, sif2.py:103-114).

Tensors on the CPU are computed on the GPU and the result returned on the
caller's device; without a GPU this raises (no CPU fallback).
"""
from __future__ import annotations

import torch

import mmb_lib as L
import pipeline as P

KEYS = ("audio", "visual", "audiovisual", "textaudio", "textvisual", "textaudiovisual")


def calc_weights(data, b_mean, b_log_sigma, mask):
    """q_mean = (x-b)/exp(2 ls), q_sigma = (x-b)^2/exp(2 ls) - 1 (mask ignored, as the reference)."""
    dev = L.require_gpu()
    home = data.device
    x = data.detach().to(dev, torch.float32)
    qm, qs = P.calc_weights(x, b_mean.detach().to(dev, torch.float32),
                            b_log_sigma.detach().to(dev, torch.float32))
    return qm.to(home), qs.to(home)


def estimate_embedding_overall_gpu2(data, masks, networks, sentence_weights, embeddings):
    dev = L.require_gpu()
    for k in KEYS:  # the reference indexes all six (sif2.py:181-184): KeyError if absent
        networks[k]
        masks[k]
    home = embeddings.device
    f32 = lambda t: t.detach().to(dev, torch.float32).contiguous()
    text = f32(data["text"])
    emb = text if embeddings is data["text"] else f32(embeddings)
    audio, visual = f32(data["audio"]), f32(data["visual"])
    sw = f32(sentence_weights)
    n, t, d = emb.shape
    a, vd = audio.shape[-1], visual.shape[-1]
    if text.shape != emb.shape or audio.shape[:2] != (n, t) or visual.shape[:2] != (n, t):
        raise RuntimeError("text, audio and visual must share [N, T] (torch.cat along features, "
                           "simplesif.py:825-830)")
    proj = P.MMB2Projection(networks, d, a, vd, t, dev)
    num, s, aux = P.mm2_stream(n, t, d, a, vd, audio, visual, text_dense=text, emb_dense=emb,
                               w_dense=sw, s_half=P.x3_supported(proj))
    if n == 1:
        # the reference squeezes the batch dim away (sif2.py:200-201) and then
        # fails in cs.norm(dim=1) (:207); keep that error behaviour
        raise IndexError("Dimension out of range (expected to be in range of [-1, 0], but got 1)")
    cs = P.mm2_project(s, num, aux, proj)
    return cs.to(home)
