"""Drop-in for the live part of `/root/reference/sif2.py` — closed-form MMB2.

* calc_weights(data, b_mean, b_log_sigma, mask)                 sif2.py:103-114
* estimate_embedding_overall_gpu2(data, masks, networks,
                                  sentence_weights, embeddings) sif2.py:164-208

Same arguments and result ([N, 300] fp32, unit rows, no PC removal).  Instead
of materialising q_mean/q_sigma [N,T,F_k] for six combinations and running
twelve matmuls, one streaming kernel reduces every utterance's frames to the
per-feature sums of x and x^2, and one fp32-MFMA GEMM against the merged
generator matrix finishes the embedding (see csrc/mm2_kernels.hip for the
algebra).  The kernel streams data['text'], data['audio'] and data['visual']
once; the four combination tensors are, at every reference call site
(simplesif.py:825-830), torch.cat of those three.  Because the result would
silently differ otherwise, the shim checks that: every combination's frame
count and feature width must equal its parts' (always), and its contents must
equal the concatenation (CHECK_CONCATENATIONS, on by default; it reads the
combination tensors once) -- a ValueError names the offending key.  The
reference ignores `masks` too (pads contribute, sif2.py:103-114).

`embeddings` / `sentence_weights` may have their own length L != T: the
reference's text term is a bmm over L (sif2.py:196-201), and --time_test on
POM passes the unaligned transcript (text_id, simplesif.py:862-871) beside the
word-aligned frames.  Then the frames are streamed with zero text weights and
the weighted text average comes from mmb_sif_wavg over the [N*L, D] rows.

Tensors on the CPU are computed on the GPU and the result returned on the
caller's device; without a GPU this raises (no CPU fallback).
"""
from __future__ import annotations

import torch

import mmb_lib as L
import pipeline as P

KEYS = ("audio", "visual", "audiovisual", "textaudio", "textvisual", "textaudiovisual")
PARTS = {"audiovisual": ("audio", "visual"), "textaudio": ("text", "audio"),
         "textvisual": ("text", "visual"), "textaudiovisual": ("text", "audio", "visual")}
CHECK_CONCATENATIONS = True


def _same(x, y) -> bool:
    if torch.equal(x, y):
        return True
    return bool(((x == y) | (torch.isnan(x) & torch.isnan(y))).all())


def check_combinations(data):
    """The combination tensors must be the concatenations the kernel assumes."""
    n, t = data["audio"].shape[:2]
    for k in ("text", "visual") + tuple(PARTS):
        x = data[k]
        if x.dim() != 3 or tuple(x.shape[:2]) != (n, t):
            raise ValueError(f"data[{k!r}] has shape {tuple(x.shape)}; every modality and "
                             f"combination must be [N={n}, T={t}, F]")
    for k, parts in PARTS.items():
        x = data[k]
        widths = [data[p].shape[-1] for p in parts]
        if x.shape[-1] != sum(widths):
            raise ValueError(f"data[{k!r}] has {x.shape[-1]} features, expected "
                             f"{' + '.join(map(str, widths))} = {sum(widths)} "
                             f"(torch.cat of {', '.join(parts)})")
        if CHECK_CONCATENATIONS:
            off = 0
            for p, w in zip(parts, widths):
                if not _same(x[..., off:off + w], data[p].to(x.device)):
                    raise ValueError(f"data[{k!r}][..., {off}:{off + w}] is not data[{p!r}]: the "
                                     f"combination tensors must be torch.cat of "
                                     f"{', '.join(parts)} (simplesif.py:825-830)")
                off += w


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
    check_combinations(data)
    home = embeddings.device
    f32 = lambda t: t.detach().to(dev, torch.float32).contiguous()
    text = f32(data["text"])
    emb = text if embeddings is data["text"] else f32(embeddings)
    audio, visual = f32(data["audio"]), f32(data["visual"])
    sw = f32(sentence_weights)
    n, t, d = text.shape
    a, vd = audio.shape[-1], visual.shape[-1]
    if emb.dim() != 3 or emb.shape[0] != n or emb.shape[-1] != d or sw.shape != emb.shape[:2]:
        raise RuntimeError(f"embeddings {tuple(emb.shape)} / sentence_weights {tuple(sw.shape)} "
                           f"do not match [N={n}, L, D={d}] / [N, L]")
    proj = P.MMB2Projection(networks, d, a, vd, t, dev)
    half = P.x3_supported(proj)
    # a few long rows (POM's splits): tokens and frames on workgroups of their own
    split = (P.split_ws(n, t, d, a, vd, dev)
             if t > 64 and 0 < n <= L.cu_count(dev) else None)
    if emb.shape[1] == t:
        num, s, aux = P.mm2_stream(n, t, d, a, vd, audio, visual, text_dense=text, emb_dense=emb,
                                   w_dense=sw, s_half=half, split=split)
    else:
        # L != T: frame sums with zero text weights, then the weighted average
        # of the L rows (a2 over the [N*L, D] rows as a table)
        l = emb.shape[1]
        num, s, aux = P.mm2_stream(n, t, d, a, vd, audio, visual, text_dense=text,
                                   emb_dense=text, w_dense=torch.zeros((n, t), device=dev),
                                   s_half=half, split=split)
        if n * l >= 2 ** 31:
            raise ValueError("N * L must be < 2^31")
        rows = torch.arange(n * l, device=dev, dtype=torch.int32).view(n, l)
        # x -> num (the a2 row), count_nonzero(w) -> aux[0], in one a2 pass
        L.call("mmb_sif_wavg", L.ptr(emb), n * l, d, L.ptr(rows), n, l, L.ptr(sw), None,
               L.ptr(num), None, L.ptr(aux[0]), None, L.stream_ptr())
        aux[1].copy_(sw.sum(-1))  # sentence_weights.sum(-1), sif2.py:186
    if n == 1:
        # the reference squeezes the batch dim away (sif2.py:200-201) and then
        # fails in cs.norm(dim=1) (:207); keep that error behaviour
        raise IndexError("Dimension out of range (expected to be in range of [-1, 0], but got 1)")
    cs = P.mm2_project(s, num, aux, proj, split=P.project_split_ws(n, proj.kp, dev))
    return cs.to(home)
