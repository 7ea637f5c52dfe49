"""Device side of the latent-optimisation objective.

The reference (`losses.py:13-95, 216-274`) scores latent sentence embeddings
with torch eager ops that materialise a [B, V, 300] cosine tensor for the word
model and a [B, T, F] tensor per modality combination for the Gaussians, every
step.  Here both terms are libmmb kernels (csrc/latent_kernels.hip) wrapped as
torch autograd Functions with hand-written backward passes:

  _WordLogProb   Z / G / h over the vocabulary (fused fp32-MFMA kernel) +
                 per-token terms;  backward: closed-form d lp / d latents
  _GaussLogProb  the Gaussian log-likelihood of every combination from
                 per-utterance masked frame sums (streamed once per split);
                 backward: closed-form d lp / d mu, d lp / d sigma
  layer_norm     the generator's LayerNorm: torch's forward, backward in ONE
                 libmmb launch (dx + deterministic dgamma / dbeta)

Gradients flow to the latents and, through torch's own autograd, to the
generator (norm + linears) and the regressor, exactly as in the reference
training loops.  Nothing here falls back to CPU: without libmmb / a GPU the
calls raise.
"""
from __future__ import annotations

import ctypes

import torch

import mmb_lib as L

MOD_BITS = {"text": 1, "audio": 2, "visual": 4}


def key_mods(key: str) -> int:
    """Modality bits of a combination key (features in text, audio, visual order)."""
    m = 0
    if key.startswith("text"):
        m |= 1
    if "audio" in key:
        m |= 2
    if "visual" in key:
        m |= 4
    if m == 0:
        raise KeyError(key)
    return m


# ------------------------------------------------------------------ word table
class WordTable:
    """A word-embedding table on device plus its row-normalised, 16-padded copy
    (torch cosine_similarity's x / max(|x|, 1e-8)), computed once."""

    def __init__(self, table: torch.Tensor):
        dev = L.require_gpu()
        self.table = table.detach().to(device=dev, dtype=torch.float32).contiguous()
        self.V, self.D = self.table.shape
        self.Dp = L.query("mmb_word_pad", self.D)
        self.wn = torch.empty((self.V, self.Dp), dtype=torch.float32, device=dev)
        L.call("mmb_word_normalize", L.ptr(self.table), self.V, self.D, L.ptr(self.wn),
               L.stream_ptr())


_table_cache: dict = {}


def word_table(word_embeddings: torch.Tensor) -> WordTable:
    """Cached WordTable for a (device) table tensor — keyed by storage and version,
    so an in-place edit of the table is noticed."""
    key = (word_embeddings.data_ptr(), tuple(word_embeddings.shape), word_embeddings._version,
           str(word_embeddings.device), word_embeddings.dtype)
    wt = _table_cache.get(key)
    if wt is None:
        if len(_table_cache) > 8:
            _table_cache.clear()
        wt = WordTable(word_embeddings)
        _table_cache[key] = wt
    return wt


class _WordLogProb(torch.autograd.Function):
    @staticmethod
    def forward(ctx, latents, table: WordTable, ids, sent_dense, w, mask, a):
        lat = latents.detach().float().contiguous()
        B, D = lat.shape
        if D != table.D:
            raise ValueError(f"latent width {D} != word-table width {table.D}")
        Lt = w.shape[1]
        dev = lat.device
        want = bool(ctx.needs_input_grad[0])
        ws = torch.empty(max(L.query("mmb_word_workspace_bytes", B, D, table.V), 16),
                         dtype=torch.uint8, device=dev)
        lp = torch.empty((B,), dtype=torch.float32, device=dev)
        state = torch.empty((B, 4), dtype=torch.float32, device=dev) if want else None
        gsum = torch.empty((B, table.Dp), dtype=torch.float32, device=dev) if want else None
        cosv = torch.empty((B, Lt), dtype=torch.float32, device=dev) if want else None
        L.call("mmb_word_logprob_forward", L.ptr(lat), B, D, L.ptr(table.wn), table.V, L.ptr(ids),
               L.ptr(table.table) if ids is not None else None, L.ptr(sent_dense), Lt, L.ptr(w),
               L.ptr(mask), float(a), int(want), L.ptr(ws), L.ptr(lp), L.ptr(state), L.ptr(gsum),
               L.ptr(cosv), L.stream_ptr())
        if want:
            ctx.save_for_backward(lat, ids, sent_dense, w, mask, state, gsum, cosv)
            ctx.table, ctx.a = table, a
        return lp

    @staticmethod
    def backward(ctx, dlp):
        lat, ids, sent_dense, w, mask, state, gsum, cosv = ctx.saved_tensors
        table = ctx.table
        B, D = lat.shape
        dlat = torch.empty_like(lat)
        L.call("mmb_word_logprob_backward", L.ptr(lat), B, D, table.V, L.ptr(ids),
               L.ptr(table.table) if ids is not None else None, L.ptr(sent_dense), w.shape[1],
               L.ptr(w), L.ptr(mask), float(ctx.a), L.ptr(state), L.ptr(gsum), L.ptr(cosv),
               L.ptr(dlp.float().contiguous()), L.ptr(dlat), L.stream_ptr())
        return dlat, None, None, None, None, None, None


def word_log_prob(latents, table: WordTable, w, mask, a, ids=None, sent_dense=None):
    """lp [B] of the angular word model (losses.py:68-95) for tokens given by
    `ids` [B, L] (rows of table) or `sent_dense` [B, L, D]; w, mask [B, L]."""
    dev = latents.device
    w = w.to(device=dev, dtype=torch.float32).contiguous()
    mask = mask.to(device=dev, dtype=torch.float32).contiguous()
    if ids is not None:
        ids = ids.to(device=dev, dtype=torch.int32).contiguous()
    if sent_dense is not None:
        sent_dense = sent_dense.detach().to(device=dev, dtype=torch.float32).contiguous()
    return _WordLogProb.apply(latents, table, ids, sent_dense, w, mask, a)


# ------------------------------------------------------------------ Gaussians
def gauss_stats(x: torch.Tensor, mask: torch.Tensor | None = None) -> torch.Tensor:
    """[N, 3, F] f64 masked frame sums of x [N, T, F] (mask [N, T, F] or None)."""
    x = x.detach().to(dtype=torch.float32).contiguous()
    N, T, F = x.shape
    st = torch.empty((N, 3, F), dtype=torch.float64, device=x.device)
    m = None
    if mask is not None:
        m = mask.detach().to(device=x.device, dtype=torch.float32).expand(N, T, F).contiguous()
    L.call("mmb_gauss_stats", L.ptr(x), L.ptr(m), N, T, F, L.ptr(st), L.stream_ptr())
    return st


def _ptr_array(ts, ctype=ctypes.c_void_p):
    return (ctype * len(ts))(*[0 if t is None else t.data_ptr() for t in ts])


class GaussStats:
    """Per-modality frame sums of one data split: text / audio / visual."""

    def __init__(self, text=None, audio=None, visual=None):
        self.stats = [text, audio, visual]
        self.fm = [0 if s is None else s.shape[2] for s in self.stats]


def _rows(t: torch.Tensor):
    """(tensor, row stride) for the strided Gaussian entry points: a [B, F]
    view with unit column stride passes as is (e.g. a key's column block of
    the generator's fused output), anything else as a contiguous copy."""
    t = t.detach()
    if t.dtype != torch.float32 or t.dim() != 2 or t.stride(1) != 1:
        t = t.float().contiguous()
    return t, t.stride(0)


class _GaussLogProb(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gs: GaussStats, idx, mods, *musig):
        K = len(mods)
        mus, ldm = zip(*[_rows(m) for m in musig[:K]])
        sigs, lds = zip(*[_rows(s) for s in musig[K:]])
        B = mus[0].shape[0]
        lp = torch.empty((K, B), dtype=torch.float32, device=mus[0].device)
        st = _ptr_array(gs.stats)
        fm = (ctypes.c_int * 3)(*gs.fm)
        md = (ctypes.c_int * K)(*mods)
        L.call("mmb_gauss_loglik_strided", st, fm, L.ptr(idx), B, K, md, _ptr_array(mus),
               (ctypes.c_int64 * K)(*ldm), _ptr_array(sigs), (ctypes.c_int64 * K)(*lds), L.ptr(lp),
               L.stream_ptr())
        ctx.gs, ctx.mods, ctx.ldm, ctx.lds = gs, mods, ldm, lds
        ctx.save_for_backward(idx, *mus, *sigs)
        return lp

    @staticmethod
    def backward(ctx, dlp):
        saved = ctx.saved_tensors
        idx = saved[0]
        K = len(ctx.mods)
        mus, sigs = saved[1:1 + K], saved[1 + K:]
        B = mus[0].shape[0]
        need_mu = ctx.needs_input_grad[3:3 + K]
        need_s = ctx.needs_input_grad[3 + K:]

        def grads(ts, lds, need):
            # one buffer for all keys, each key's block at its input's offset
            # and row stride (the layout of the generator's fused output), so
            # the gradients reach the split / linear backward without copies
            if not any(need):
                return [None] * K
            base = ts[0]
            same = all(t.stride(0) == lds[0] and t.untyped_storage().data_ptr() ==
                       base.untyped_storage().data_ptr() for t in ts)
            if same:
                # one slot per key only if the keys' column blocks are disjoint
                # (one tensor or overlapping views passed for two keys would
                # otherwise share a slot: the kernel keeps one key's gradient
                # and autograd adds it once per key)
                blocks = sorted((t.storage_offset(), t.shape[1]) for t, n in zip(ts, need) if n)
                same = all(o0 + w0 <= o1 for (o0, w0), (o1, _) in zip(blocks, blocks[1:]))
            if not same:
                return [torch.empty_like(t) if n else None for t, n in zip(ts, need)]
            lo = min(t.storage_offset() for t in ts)
            width = max(t.storage_offset() - lo + t.shape[1] for t in ts)
            buf = torch.empty((B, lds[0]), dtype=torch.float32, device=base.device)
            return [buf[:, t.storage_offset() - lo:t.storage_offset() - lo + t.shape[1]] if n
                    else None for t, n in zip(ts, need)] if width <= lds[0] else \
                [torch.empty_like(t) if n else None for t, n in zip(ts, need)]

        dmu = grads(mus, ctx.ldm, need_mu)
        dsg = grads(sigs, ctx.lds, need_s)
        ldm = [d.stride(0) if d is not None else l for d, l in zip(dmu, ctx.ldm)]
        lds = [d.stride(0) if d is not None else l for d, l in zip(dsg, ctx.lds)]
        # (a key's gradient must share its input's row stride: the kernel walks both with one)
        assert all(a == b for a, b in zip(ldm, ctx.ldm)) and all(a == b for a, b in zip(lds, ctx.lds))
        gs = ctx.gs
        L.call("mmb_gauss_backward_strided", _ptr_array(gs.stats), (ctypes.c_int * 3)(*gs.fm),
               L.ptr(idx), B, K, (ctypes.c_int * K)(*ctx.mods), _ptr_array(mus),
               (ctypes.c_int64 * K)(*ctx.ldm), _ptr_array(sigs), (ctypes.c_int64 * K)(*ctx.lds),
               L.ptr(dlp.float().contiguous()), _ptr_array(dmu), _ptr_array(dsg), L.stream_ptr())
        return (None, None, None, *dmu, *dsg)


def gauss_log_prob(gs: GaussStats, keys, mus, sigmas, idx=None):
    """lp [K, B]: get_normal_log_prob (losses.py:13-33) of every combination in
    `keys`, mus/sigmas [B, F_k], from the frame sums of rows idx [B] (or 0..B)."""
    mods = [key_mods(k) for k in keys]
    if idx is not None:
        idx = idx.to(device=mus[0].device, dtype=torch.int64).contiguous()
    return _GaussLogProb.apply(gs, idx, mods, *mus, *sigmas)


class _LayerNorm(torch.autograd.Function):
    """nn.LayerNorm over the last dim (reference models.py:163-164); the forward
    is torch's (native_layer_norm, which also returns the row mean / rstd), the
    backward is `mmb_layer_norm_backward` — one launch where torch's takes two,
    its column reduction ~21 us for a 64 x 300 batch (profiles/r03_latent)."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        D = x.shape[-1]
        x2 = x.reshape(-1, D).contiguous()
        y, mean, rstd = torch.native_layer_norm(x2, [D], weight, bias, eps)
        ctx.save_for_backward(x2, mean, rstd, weight)
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, mean, rstd, w = ctx.saved_tensors
        N, D = x2.shape
        dy2 = dy.reshape(N, D).contiguous()
        dx = torch.empty_like(x2)
        dw = torch.empty_like(w) if ctx.needs_input_grad[1] else None
        db = torch.empty_like(w) if ctx.needs_input_grad[2] else None
        L.call("mmb_layer_norm_backward", L.ptr(dy2), L.ptr(x2), L.ptr(mean), L.ptr(rstd),
               L.ptr(w), N, D, L.ptr(dx), L.ptr(dw), L.ptr(db), L.stream_ptr())
        return dx.view(ctx.shape), dw, db, None


def layer_norm(x, weight, bias, eps):
    """LayerNorm with the libmmb backward (f32 device tensors, affine)."""
    for t in (x, weight, bias):
        if t.dtype != torch.float32 or not t.is_cuda:
            raise L.MMBError("layer_norm takes f32 device tensors")
    return _LayerNorm.apply(x, weight.contiguous(), bias.contiguous(), eps)
