"""CPU restatement of the closed-form MMB2 estimate (a7/a8) — TEST INFRASTRUCTURE ONLY.

Follows `/root/reference/sif2.py:103-114` (calc_weights) and `:164-208`
(estimate_embedding_overall_gpu2), restated in numpy so it can run in float64
(the parity target) or float32 (the reference's own arithmetic).
"""
from __future__ import annotations

import numpy as np

KEYS = ("audio", "visual", "audiovisual", "textaudio", "textvisual", "textaudiovisual")


def calc_weights(data, b_mean, b_log_sigma):
    """sif2.py:103-114 — the mask argument is ignored by the reference (pads count)."""
    b_mean = b_mean.reshape((1, 1, -1))
    b_log_sigma = b_log_sigma.reshape((1, 1, -1))
    q_mean = (data - b_mean) / np.exp(2 * b_log_sigma)
    q_sigma = (data - b_mean) ** 2 / np.exp(2 * b_log_sigma) - 1.0
    return q_mean, q_sigma


def concat_inputs(text, audio, visual):
    """The 7 data tensors the callers build (simplesif.py:820-830)."""
    return {"text": text, "audio": audio, "visual": visual,
            "audiovisual": np.concatenate([audio, visual], -1),
            "textaudio": np.concatenate([text, audio], -1),
            "textvisual": np.concatenate([text, visual], -1),
            "textaudiovisual": np.concatenate([text, audio, visual], -1)}


def estimate_embedding_overall_gpu2(data, params, sentence_weights, embeddings, dtype=np.float64):
    """sif2.py:164-208.

    params: {key: (W_mu [F,D], b_mu [F], W_ls [F,D], b_ls [F])} as numpy.
    Keys are visited in the fixed order of :167-174; total weight is the sum of
    sentence weights plus every q_mean and q_sigma element (:186-188); cs is
    the weighted text average plus sum_k sum_t (q/total) @ W_k (:200-205), then
    row-L2-normalised (:207).  No PC removal.
    """
    c = lambda a: np.asarray(a, dtype=dtype)
    qm, qs = {}, {}
    for k in KEYS:
        Wm, bm, Wl, bl = params[k]
        qm[k], qs[k] = calc_weights(c(data[k]), c(bm), c(bl))
    sw = c(sentence_weights)
    total = sw.sum(-1) + sum(qm[k].sum(-1).sum(-1) for k in KEYS)
    total = total + sum(qs[k].sum(-1).sum(-1) for k in KEYS)
    total = total.reshape((-1, 1, 1))
    cs = np.einsum("nt,ntd->nd", sw / total.reshape((-1, 1)), c(embeddings))
    for k in KEYS:
        Wm, bm, Wl, bl = params[k]
        cs = cs + np.matmul(qm[k] / total, c(Wm)).sum(axis=1)
        cs = cs + np.matmul(qs[k] / total, c(Wl)).sum(axis=1)
    cs = cs / np.linalg.norm(cs, axis=1, keepdims=True)
    return cs


def params_from_module(gen):
    """{key: (W_mu, b_mu, W_ls, b_ls)} numpy f32 from an AudioVisualGeneratorMultimodal."""
    out = {}
    for k, m in gen.embed2out.items():
        out[k] = tuple(t.detach().cpu().numpy() for t in (m["mu"].weight, m["mu"].bias,
                                                           m["log_sigma"].weight, m["log_sigma"].bias))
    return out


def row_rel_err(y, yref):
    """SURVEY §8d parity metric: max_j |y - yref| / max_j |yref| per row, max over rows."""
    y = np.asarray(y, np.float64)
    yref = np.asarray(yref, np.float64)
    return float((np.abs(y - yref).max(axis=1) / np.abs(yref).max(axis=1)).max())
