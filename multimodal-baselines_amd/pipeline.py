"""Device-resident hot path: SIF (a1-a5) and closed-form MMB2 (a6-a8) on HBM tensors.

Every function here takes and returns torch device tensors and calls libmmb
through its C ABI on the current stream; nothing is synchronised.  The
reference-signature mirrors (`sif_functions.py`, `sif.py`, `sif2.py`) and
`bench.py` are thin layers over these.

Data layout in HBM (one utterance per row, row-major, fp32 unless noted):
  table [V, D], wtab [V] (f32 rounding of the f64 SIF weights), ids [N, L] int32,
  audio [N, T, A], visual [N, T, Vd]                                  (inputs)
  x [N, D]     a2 rows (weighted text sum / count)   s [N, Kp] frame sums   aux [3, N]
  G [D, D] f64 Gram   pc [npc, D] f64                                  (intermediates)
  sif [N, D] (f32 or f64)   mmb2 [N, D]                               (outputs)
"""
from __future__ import annotations

import os

import numpy as np
import torch

import mmb_lib as L
from models import MMB2_KEYS

N_OVERSAMPLES = 10  # sklearn randomized_svd default (extmath.py:535)
N_ITER = 7          # TruncatedSVD(n_iter=7), sif_functions.py:65
PC_SEED = 0         # random_state=0, sif_functions.py:65

_omega_cache: dict = {}


def omega(rows: int, k: int, device) -> torch.Tensor:
    """RandomState(0).normal(size=(rows, k)) as f64 on `device` (cached)."""
    key = (rows, k, str(device))
    t = _omega_cache.get(key)
    if t is None:
        host = L.host_randn(PC_SEED, rows * k).reshape(rows, k)
        t = torch.from_numpy(host).to(device)
        if len(_omega_cache) > 16:
            _omega_cache.clear()
        _omega_cache[key] = t
    return t


def narrow_ids(ids: torch.Tensor) -> torch.Tensor:
    """int64 reference ids -> int32 device ids (range-checked)."""
    if ids.dtype == torch.int32:
        return ids.contiguous()
    if ids.numel():
        lo, hi = int(ids.min()), int(ids.max())
        if lo < -(2 ** 31) or hi >= 2 ** 31:
            raise IndexError("token id out of int32 range")
    return ids.to(torch.int32).contiguous()


MAX_NPC = 16 - N_OVERSAMPLES  # the device solver keeps the k = npc + 10 block in 16 columns


def check_npc(npc: int):
    if not 1 <= npc <= MAX_NPC:
        raise ValueError(f"npc={npc}: the device PC solver supports 1 <= npc <= {MAX_NPC} "
                         f"(randomized-SVD block npc + {N_OVERSAMPLES} <= 16 columns)")


def check_flag(flag: torch.Tensor, V: int, zero_weights: bool = False):
    """Raise like the reference for what the kernels reported in `flag`:
    IndexError for an id >= V (numpy fancy indexing); with `zero_weights`,
    ValueError for an utterance whose weights are all 0 -- its a2 row is
    0/0 = NaN (sif_functions.py:55) and the reference's TruncatedSVD rejects
    the split (sklearn check_array: "Input X contains NaN")."""
    check_flag_bits(int(flag.item()), V, zero_weights)


def check_flag_bits(f: int, V: int, zero_weights: bool = False):
    """check_flag on flag bits already read back."""
    if f & L.MMB_FLAG_SYNC_TIMEOUT:
        raise RuntimeError("a bounded in-kernel hand-over timed out (mmb_mm2_stream_project's "
                           "streaming / projecting waves, or mmb_pc_solve_mc's workgroups); "
                           "the step's MMB2 rows or PC are invalid")
    if f & L.MMB_FLAG_ID_RANGE:
        raise IndexError(f"token id out of bounds for a vocabulary of size {V}")
    if zero_weights and f & L.MMB_FLAG_ZERO_WEIGHTS:
        raise ValueError("Input X contains NaN: an utterance whose SIF weights are all 0 has a "
                         "0/0 weighted average (sif_functions.py:55), which the reference's "
                         "TruncatedSVD rejects (sif_functions.py:65-67)")


# status word of a checked step: the flag bits | PC_NONFINITE (FusedStep.status)
PC_NONFINITE = 1 << 16


# ------------------------------------------------------------------ a1
def seq2weight(seq32: torch.Tensor, sel: torch.Tensor | None, wtab64: torch.Tensor,
               flag: torch.Tensor | None = None) -> torch.Tensor:
    n, l = seq32.shape
    w = torch.empty((n, l), dtype=torch.float32, device=seq32.device)
    L.call("mmb_seq2weight", L.ptr(seq32), L.ptr(sel), n, l, L.ptr(wtab64), wtab64.numel(),
           L.ptr(w), L.ptr(flag), L.stream_ptr())
    return w


# ------------------------------------------------------------------ a1+a2
def weighted_sum(table: torch.Tensor, ids32: torch.Tensor, w: torch.Tensor | None = None,
                 wtab32: torch.Tensor | None = None, flag: torch.Tensor | None = None,
                 x_out: bool = False):
    """Returns (num [N,D], cnt [N]) or x [N,D] (= num/cnt) if x_out."""
    n, l = ids32.shape
    V, D = table.shape
    dev = table.device
    if x_out:
        x = torch.empty((n, D), dtype=torch.float32, device=dev)
        L.call("mmb_sif_wavg", L.ptr(table), V, D, L.ptr(ids32), n, l, L.ptr(w), L.ptr(wtab32),
               L.ptr(x), None, None, L.ptr(flag), L.stream_ptr())
        return x
    num = torch.empty((n, D), dtype=torch.float32, device=dev)
    cnt = torch.empty((n,), dtype=torch.float32, device=dev)
    L.call("mmb_sif_wavg", L.ptr(table), V, D, L.ptr(ids32), n, l, L.ptr(w), L.ptr(wtab32),
           None, L.ptr(num), L.ptr(cnt), L.ptr(flag), L.stream_ptr())
    return num, cnt


# ------------------------------------------------------------------ a3
class GramWorkspace:
    """Scratch for mmb_gram sized for up to `n` rows (re-used across calls)."""

    def __init__(self, n: int, d: int, device):
        nbytes = L.query("mmb_gram_workspace_bytes", n, d)
        self.buf = torch.empty(max(nbytes, 8), dtype=torch.uint8, device=device)
        self.n, self.d = n, d

    def fits(self, n, d):
        return L.query("mmb_gram_workspace_bytes", n, d) <= self.buf.numel()


def gram(num: torch.Tensor, cnt: torch.Tensor | None, G: torch.Tensor | None = None,
         accumulate: bool = False, ws: GramWorkspace | None = None) -> torch.Tensor:
    n, d = num.shape
    if G is None:
        G = torch.empty((d, d), dtype=torch.float64, device=num.device)
    if ws is None or not ws.fits(n, d):
        ws = GramWorkspace(n, d, num.device)
    L.call("mmb_gram", L.ptr(num), L.ptr(cnt), n, d, L.ptr(G), int(accumulate), L.ptr(ws.buf),
           L.stream_ptr())
    return G


def colmax(x: torch.Tensor, out: torch.Tensor | None = None, accumulate: bool = False):
    """Column bounds max_i |x[i, j]| as float bits (int32 view of uint32) for
    the int8 Gram (mmb_colmax)."""
    n, d = x.shape
    if out is None:
        out = torch.empty((d,), dtype=torch.int32, device=x.device)
    L.call("mmb_colmax", L.ptr(x), n, d, L.ptr(out), int(accumulate), L.stream_ptr())
    return out


def gram_i8(x: torch.Tensor, cmax: torch.Tensor, G: torch.Tensor | None = None,
            accumulate: bool = False, ws: GramWorkspace | None = None) -> torch.Tensor:
    """G = x^T x on the int8 matrix pipe (mmb_gram_i8): 33-bit fixed point per
    column bound, ~1e-10 relative to the exact f64 Gram."""
    n, d = x.shape
    if G is None:
        G = torch.empty((d, d), dtype=torch.float64, device=x.device)
    if ws is None or not ws.fits(n, d):
        ws = GramWorkspace(n, d, x.device)
    L.call("mmb_gram_i8", L.ptr(x), L.ptr(cmax), n, d, L.ptr(G), int(accumulate), L.ptr(ws.buf),
           L.stream_ptr())
    return G


def xt_omega(num, cnt, omega_rows: torch.Tensor) -> torch.Tensor:
    n, d = num.shape
    k = omega_rows.shape[1]
    z0 = torch.empty((d, k), dtype=torch.float64, device=num.device)
    L.call("mmb_xt_omega", L.ptr(num), L.ptr(cnt), n, d, L.ptr(omega_rows), k, L.ptr(z0),
           L.stream_ptr())
    return z0


def pc_start_block(n_total: int, d: int, npc: int, device, num=None, cnt=None, row0: int = 0,
                   n_total_rows_omega: int | None = None):
    """Z0 of sklearn's randomized SVD.  Direct branch: Omega [d,k].  Transposed
    branch (n_total < d): X^T Omega_n for this shard's rows [row0, row0+n)."""
    check_npc(npc)
    k = npc + N_OVERSAMPLES
    if n_total >= d:
        return omega(d, k, device), False
    om = omega(n_total, k, device)[row0:row0 + num.shape[0]].contiguous()
    return xt_omega(num, cnt, om), True


PC_SOLVE_MC_MAX_D = 320  # mmb_pc_solve_mc: ceil(d / 16) workgroups, k <= 16
_solve_ws: dict = {}


def solve_workspace(d: int, device) -> torch.Tensor:
    """Scratch of mmb_pc_solve_mc (the tiles exchanged between its
    workgroups), one per (d, device, current stream): a call owns it until
    it completes, and calls on one stream are ordered."""
    key = (d, str(device), L.stream_ptr())
    ws = _solve_ws.get(key)
    if ws is None:  # zeroed once: a completed solve leaves its control words zero
        ws = torch.zeros(L.query("mmb_pc_solve_mc_ws_bytes", d), dtype=torch.uint8, device=device)
        if len(_solve_ws) > 16:
            _solve_ws.clear()
        _solve_ws[key] = ws
    return ws


def pc_solve(G: torch.Tensor, z0: torch.Tensor, npc: int, transposed: bool,
             n_iter: int = N_ITER, out: torch.Tensor | None = None,
             flag: torch.Tensor | None = None, ws: torch.Tensor | None = None) -> torch.Tensor:
    """sklearn's randomized-SVD components from the Gram (a3's solve).  d <=
    320: the multi-workgroup solver (mmb_pc_solve_mc); larger d: one
    workgroup.  A hand-over timeout of the multi-workgroup solver leaves NaN
    in the PC and sets MMB_FLAG_SYNC_TIMEOUT in `flag`: a caller that passes
    its own flag (FusedStep, graph-capturable) checks it later; without one,
    this call checks a flag of its own and raises here (one host sync)."""
    d = G.shape[0]
    k = z0.shape[1]
    pc = out if out is not None else torch.empty((npc, d), dtype=torch.float64, device=G.device)
    if d <= PC_SOLVE_MC_MAX_D and k <= 16:
        if ws is None:
            ws = solve_workspace(d, G.device)
        own = flag is None
        if own:
            flag = torch.zeros(1, dtype=torch.int32, device=G.device)
        L.call("mmb_pc_solve_mc", L.ptr(G), d, L.ptr(z0), k, npc, n_iter, int(transposed),
               L.ptr(pc), L.ptr(ws), L.ptr(flag), L.stream_ptr())
        if own and int(flag.item()) & L.MMB_FLAG_SYNC_TIMEOUT:
            ws[:16].zero_()  # an aborted solve leaves its control words set
            raise RuntimeError("mmb_pc_solve_mc: a bounded hand-over between the solver's "
                               "workgroups timed out; the PC is invalid (NaN)")
    else:
        L.call("mmb_pc_solve", L.ptr(G), d, L.ptr(z0), k, npc, n_iter, int(transposed), L.ptr(pc),
               L.stream_ptr())
    return pc


# ------------------------------------------------------------------ a4
def remove_pc(num, cnt, pc: torch.Tensor, out_dtype=torch.float32, out=None) -> torch.Tensor:
    n, d = num.shape
    if out is None:
        out = torch.empty((n, d), dtype=out_dtype, device=num.device)
    o32 = L.ptr(out) if out.dtype == torch.float32 else None
    o64 = L.ptr(out) if out.dtype == torch.float64 else None
    L.call("mmb_pc_remove", L.ptr(num), L.ptr(cnt), n, d, L.ptr(pc), pc.shape[0], o32, o64,
           L.stream_ptr())
    return out


# ------------------------------------------------------------------ a3/a4 on float64 X
def pc_f64(x64: torch.Tensor, npc: int) -> torch.Tensor:
    """PC of a float64 X [n, d] that is not f32-representable (the numpy
    drop-ins' general input): Gram, start block and solve all read f64 rows."""
    check_npc(npc)
    n, d = x64.shape
    k = npc + N_OVERSAMPLES
    G = torch.empty((d, d), dtype=torch.float64, device=x64.device)
    ws = GramWorkspace(n, d, x64.device)
    L.call("mmb_gram_f64", L.ptr(x64), n, d, L.ptr(G), 0, L.ptr(ws.buf), L.stream_ptr())
    if n >= d:
        z0, transposed = omega(d, k, x64.device), False
    else:
        z0, transposed = torch.empty((d, k), dtype=torch.float64, device=x64.device), True
        L.call("mmb_xt_omega_f64", L.ptr(x64), n, d, L.ptr(omega(n, k, x64.device)), k,
               L.ptr(z0), L.stream_ptr())
    return pc_solve(G, z0, npc, transposed)


def remove_pc_f64(x64: torch.Tensor, pc: torch.Tensor) -> torch.Tensor:
    n, d = x64.shape
    out = torch.empty((n, d), dtype=torch.float64, device=x64.device)
    L.call("mmb_pc_remove_f64", L.ptr(x64), n, d, L.ptr(pc), pc.shape[0], L.ptr(out),
           L.stream_ptr())
    return out


class DeviceOps:
    """The libmmb kernels global_pc() composes (tests substitute CPU doubles)."""

    gram = staticmethod(lambda num, cnt, G=None, ws=None: gram(num, cnt, G, ws=ws))
    omega = staticmethod(omega)
    xt_omega = staticmethod(xt_omega)
    pc_solve = staticmethod(pc_solve)


def global_pc(num, cnt, npc: int, n_total: int, row0: int = 0, allreduce=None, ops=DeviceOps,
              G=None, ws=None):
    """The PC of ALL utterances across ranks (a3), from this rank's rows
    [row0, row0 + n) of X = num / cnt.

    Only the Gram (d x d f64) — and, in sklearn's transposed branch (fewer
    utterances than features), the start block X^T Omega (d x k) — cross
    ranks, each as one all-reduce (sum).  Every rank then runs the same
    deterministic solve, so the PC is identical everywhere with no broadcast.
    """
    n, d = num.shape
    check_npc(npc)
    k = npc + N_OVERSAMPLES
    G = ops.gram(num, cnt, G, ws)
    if n_total >= d:
        z0, transposed = ops.omega(d, k, num.device), False
    else:
        om = ops.omega(n_total, k, num.device)[row0:row0 + n].contiguous()
        z0, transposed = ops.xt_omega(num, cnt, om), True
    if allreduce is not None:
        allreduce(G)
        if transposed:
            allreduce(z0)
    return ops.pc_solve(G, z0, npc, transposed)


def sif_embeddings(table, ids, wtab32=None, w=None, npc: int = 1, out_dtype=torch.float32,
                   check_ids: bool = True, allreduce=None, n_total=None, row0: int = 0):
    """a1-a5 fused on device: weighted average, Gram (+ optional all-reduce
    across ranks), randomized-SVD PC, removal.  Returns (emb [N,D], pc)."""
    ids32 = narrow_ids(ids)
    flag = torch.zeros(1, dtype=torch.int32, device=table.device)
    num, cnt = weighted_sum(table, ids32, w=w, wtab32=wtab32, flag=flag)
    n_total = num.shape[0] if n_total is None else n_total
    pc = global_pc(num, cnt, npc, n_total, row0, allreduce)
    out = remove_pc(num, cnt, pc, out_dtype)
    if not check_ids:  # the id-range bit is then not the caller's concern
        flag.bitwise_and_(~L.MMB_FLAG_ID_RANGE)
    check_flag(flag, table.shape[0], zero_weights=True)
    check_pc_finite(pc)
    return out, pc


def check_pc_finite(pc: torch.Tensor):
    """A NaN row on ANY rank reaches every rank's PC through the Gram
    all-reduce: checking the PC makes every rank raise, not only the one that
    holds the row."""
    if not bool(torch.isfinite(pc).all()):
        raise ValueError("Input X contains NaN or infinity: the split's Gram is not finite "
                         "(an all-zero-weight utterance on some rank, or non-finite inputs), "
                         "which the reference's TruncatedSVD rejects (sif_functions.py:65-67)")


# ------------------------------------------------------------------ a7 / a8
def calc_weights(x: torch.Tensor, b_mean: torch.Tensor, b_log_sigma: torch.Tensor):
    x = x.contiguous()
    f = x.shape[-1]
    qm = torch.empty_like(x)
    qs = torch.empty_like(x)
    L.call("mmb_calc_weights", L.ptr(x), x.numel() // f, f, L.ptr(b_mean.contiguous()),
           L.ptr(b_log_sigma.contiguous()), L.ptr(qm), L.ptr(qs), L.stream_ptr())
    return qm, qs


def mm2_dims(d, a, vd):
    return L.query("mmb_mm2_k", d, a, vd), L.query("mmb_mm2_ldw", d)


class MMB2Projection:
    """Merged [Kp, ldw] projection of the six generators (sif2.py:167-205)."""

    def __init__(self, networks: dict, d: int, a: int, vd: int, t: int, device):
        self.d, self.a, self.vd, self.t = d, a, vd, t
        self.kp, self.ldw = mm2_dims(d, a, vd)
        self.wm = torch.empty((self.kp, self.ldw), dtype=torch.float32, device=device)
        self.c0 = torch.empty((self.ldw,), dtype=torch.float32, device=device)
        nbytes = L.query("mmb_mm2_split_bytes", d, a, vd)
        self.wsplit = torch.empty((nbytes + 15) // 16 * 16, dtype=torch.uint8, device=device)
        self.device = device
        self.networks = {k: networks[k] for k in MMB2_KEYS}  # KeyError like sif2.py:182
        self.refresh()

    def _live(self):
        """The generators' current parameter tensors (w_mu, b_mu, w_ls, b_ls per key)."""
        return [(mu.weight, mu.bias, ls.weight, ls.bias)
                for mu, ls in (self.networks[k] for k in MMB2_KEYS)]

    def _versions(self):
        # storage address + version counter of every parameter: an optimiser
        # step (in place) bumps the counter, `p.data = t` moves the address
        # (and of the word / weight tables behind the text cache)
        live = [t for ps in self._live() for t in ps]
        if getattr(self, "text_src", None) is not None:
            live += list(self.text_src)
        return tuple((t.data_ptr(), t._version) for t in live)

    def invalidate(self):
        """Force a re-merge at the next refresh_if_changed(): needed after
        writes that neither bump a parameter's version counter nor move its
        storage (e.g. `p.data.copy_(...)`, which bypasses autograd's counter)."""
        self._seen = None

    def refresh(self):
        self.params = [tuple(p.detach().to(device=self.device, dtype=torch.float32).contiguous()
                             for p in ps) for ps in self._live()]
        arr = lambda i: (ctypes_ptr_array([p[i].data_ptr() for p in self.params]))
        L.call("mmb_mm2_prepare", arr(0), arr(1), arr(2), arr(3), self.d, self.a, self.vd, self.t,
               L.ptr(self.wm), self.ldw, L.ptr(self.c0), L.ptr(self.wsplit), L.stream_ptr())
        if getattr(self, "wpieces", None) is not None:
            L.call("mmb_mm2_split_pieces", L.ptr(self.wm), self.d, self.a, self.vd, self.ldw,
                   L.ptr(self.wpieces), L.stream_ptr())
        if getattr(self, "text_cache", None) is not None:
            self._build_text_cache()
        self._seen = self._versions()

    def enable_text_cache(self, table: torch.Tensor, wtab32: torch.Tensor):
        """Also keep the text cache of the narrow fused step
        (mmb_mm2_text_cache: P = E Wm_t1 + E^2 Wm_t2 per word, f64 rounded
        once, and the hot-word ranks), rebuilt with every re-merge and when
        the word or weight table changes.  The narrow fused kernel reads the
        token weights from the cache's own copy, so the cache is keyed on BOTH
        tensors (identity here, storage address + version counter in
        refresh_if_changed); writes into them that bump neither (raw-pointer
        writes by other libmmb kernels, `t.data.copy_`) need invalidate()."""
        src = getattr(self, "text_src", None)
        if (getattr(self, "text_cache", None) is None or src[0] is not table
                or src[1] is not wtab32):
            self.enable_pieces()
            V = table.shape[0]
            nbytes = (L.query("mmb_mm2_text_cache_bytes", V, self.d) + 15) // 16 * 16
            old = getattr(self, "text_cache", None)
            if old is None or old.numel() != nbytes or old.device != table.device:
                self.text_cache = torch.empty(nbytes, dtype=torch.uint8, device=table.device)
            self.text_src = (table, wtab32)
            self._build_text_cache()
            self._seen = self._versions()

    def _build_text_cache(self):
        table, wtab32 = self.text_src
        L.call("mmb_mm2_text_cache", L.ptr(table), table.shape[0], self.d, L.ptr(wtab32),
               L.ptr(self.wm), self.ldw, L.ptr(self.text_cache), L.stream_ptr())

    def enable_pieces(self):
        """Also keep the piece-ordered split of wm (mmb_mm2_split_pieces), the
        B operand of the fused stream + projection kernel."""
        if getattr(self, "wpieces", None) is None:
            nbytes = L.query("mmb_mm2_split_pieces_bytes", self.d, self.a, self.vd)
            self.wpieces = torch.empty((nbytes + 15) // 16 * 16, dtype=torch.uint8,
                                       device=self.wm.device)
            L.call("mmb_mm2_split_pieces", L.ptr(self.wm), self.d, self.a, self.vd, self.ldw,
                   L.ptr(self.wpieces), L.stream_ptr())

    def refresh_if_changed(self) -> bool:
        """Re-merge only when a generator parameter changed since the last
        merge (torch's version counters -- an optimiser step bumps them -- or
        a parameter's storage moved), so a step over a new batch with the same
        weights skips the five prepare launches.  Writes through `p.data`
        bump no counter: call invalidate() after them.  Returns whether it
        re-merged."""
        if getattr(self, "_seen", None) == self._versions():
            return False
        self.refresh()
        return True


def ctypes_ptr_array(ptrs):
    import ctypes

    return (ctypes.c_void_p * len(ptrs))(*ptrs)


def split_parts(n: int, t: int) -> int:
    """Token / frame ranges per utterance of the few-long-rows stream path
    (mmb_mm2_stream_split_parts: a text, an audio and a visual workgroup per
    range, about one workgroup per CU in all)."""
    return int(L.query("mmb_mm2_stream_split_parts", n, t))


def split_ws(n: int, t: int, d: int, a: int, vd: int, device, parts: int = 0) -> torch.Tensor:
    """Scratch of mmb_mm2_stream_split (its per-range partial rows)."""
    nb = int(L.query("mmb_mm2_stream_split_ws_bytes", n, t, d, a, vd, parts))
    return torch.empty(max(nb, 16), dtype=torch.uint8, device=device)


def mm2_stream(n, t, d, a, vd, audio, visual, ids32=None, table=None, wtab32=None,
               text_dense=None, emb_dense=None, w_dense=None, flag=None, out=None,
               s_half: bool = True, colmax=None, colmax_ws=None, split=None, parts: int = 0):
    """a6-a8 frame sums.  Returns (x, s, aux): x [n, d] the a2 rows (weighted
    text sum / count_nonzero(w)), aux [3, n] (count, total weight, row scale).
    s_half=True (default) writes s as fp16 [n, 2*kp] (hi | lo planes of the
    row-scaled sums, the x3 projection's A operand); s_half=False writes fp32
    [n, kp] for the fp32-MFMA projection.  With `colmax` ([d] int32) and
    `colmax_ws` (mmb_mm2_colmax_ws_bytes) the kernel also writes the column
    bounds max_i |x[i, j]| (float bits) for mmb_gram_i8.  With `split` (a
    split_ws scratch) every utterance's tokens / frames are cut into `parts`
    ranges (0: split_parts) summed by their own workgroups, then added in
    part order (mmb_mm2_stream_split: a few long rows, POM's splits)."""
    kp, _ = mm2_dims(d, a, vd)
    dev = audio.device
    if out is None:
        out = (torch.empty((n, d), dtype=torch.float32, device=dev),
               s_buffer(n, kp, s_half, dev),
               torch.empty((3, n), dtype=torch.float32, device=dev))
    num, s, aux = out
    if s.dtype != (torch.float16 if s_half else torch.float32):
        raise L.MMBError("s buffer dtype does not match s_half")
    V = table.shape[0] if table is not None else 0
    _check_colmax_ws(colmax_ws, d)
    if split is not None:
        L.call("mmb_mm2_stream_split", L.ptr(ids32), L.ptr(table), V, L.ptr(wtab32),
               L.ptr(text_dense), L.ptr(emb_dense), L.ptr(w_dense), L.ptr(audio), L.ptr(visual),
               n, t, d, a, vd, L.ptr(num), L.ptr(s), int(s_half), L.ptr(aux), L.ptr(flag),
               L.ptr(colmax), L.ptr(colmax_ws), int(parts), L.ptr(split),
               split.numel() * split.element_size(), L.stream_ptr())
        return num, s, aux
    L.call("mmb_mm2_stream", L.ptr(ids32), L.ptr(table), V, L.ptr(wtab32), L.ptr(text_dense),
           L.ptr(emb_dense), L.ptr(w_dense), L.ptr(audio), L.ptr(visual), n, t, d, a, vd,
           L.ptr(num), L.ptr(s), int(s_half), L.ptr(aux), L.ptr(flag), L.ptr(colmax),
           L.ptr(colmax_ws), L.stream_ptr())
    return num, s, aux


# Narrowest frame row (floats) for which the fused stream + projection step is
# the default: its 4 streaming waves per CU load every modality row as 16-B
# columns on 64 lanes, so a frame row under 256 floats leaves lanes idle and
# costs as many load round trips as a full one, while the two-kernel step's
# stream kernel (one wave per utterance, no LDS ring) keeps more loads in
# flight.  Measured (r03t, tools/step_ab.py, 500k-1M utterances, ms per
# step fused / two-kernel): A = 76, Vd = 48 at T = 20 / 40 / 64: 12.3 / 8.0,
# 8.7 / 5.8, 11.9 / 7.8 (V = 3016); 6.6 / 4.2 (V = 400k, T = 20); A = Vd = 300
# at T = 30 / 40: 10.3 / 11.0, 12.2 / 12.7 (V = 400k).
FUSED_MIN_FRAME = 256


def fused_pays(a: int, vd: int) -> bool:
    return min(a, vd) >= FUSED_MIN_FRAME


def stream_project_supported(t: int, d: int, a: int, vd: int) -> bool:
    """Shapes the fused stream + projection kernel takes (t <= 64 frames,
    256 <= d < 320, widths % 4, k <= 1920): the bench / MOSI-like configs."""
    return bool(L.query("mmb_mm2_stream_project_supported", t, d, a, vd))


def narrow_fused_supported(t: int, d: int, a: int, vd: int, v: int) -> bool:
    """Shapes of the narrow fused kernel (mmb_mm2_stream_project_narrow):
    MOSI-like frame widths (4..128, kq(A) + kq(Vd) <= 256), 256 < d < 304,
    t <= 64, a word table of <= 16384 rows (its text cache)."""
    return bool(L.query("mmb_mm2_stream_project_narrow_supported", t, d, a, vd, v))


def mm2_stream_project_narrow(n, t, d, a, vd, audio, visual, proj: "MMB2Projection", ids32,
                              table, wtab32, flag=None, out=None, colmax=None, colmax_ws=None):
    """a1-a8 at narrow frame widths in ONE kernel (mmb_mm2_stream_project_narrow):
    x, aux, the MMB2 rows (and the column bounds).  Returns (x, aux, mmb2)."""
    dev = audio.device
    if out is None:
        out = (torch.empty((n, d), dtype=torch.float32, device=dev),
               torch.empty((3, n), dtype=torch.float32, device=dev),
               torch.empty((n, d), dtype=torch.float32, device=dev))
    num, aux, mmb2 = out
    proj.enable_text_cache(table, wtab32)
    _check_colmax_ws(colmax_ws, d)
    L.call("mmb_mm2_stream_project_narrow", L.ptr(ids32), L.ptr(table), table.shape[0],
           L.ptr(wtab32), L.ptr(proj.text_cache), L.ptr(audio), L.ptr(visual), n, t, d, a, vd,
           L.ptr(proj.wpieces), L.ptr(proj.c0), L.ptr(num), L.ptr(aux), L.ptr(mmb2), L.ptr(flag),
           L.ptr(colmax), L.ptr(colmax_ws), L.stream_ptr())
    return num, aux, mmb2


def mm2_stream_project(n, t, d, a, vd, audio, visual, proj: "MMB2Projection", ids32=None,
                       table=None, wtab32=None, text_dense=None, w_dense=None, flag=None,
                       out=None, colmax=None, colmax_ws=None):
    """a6-a8 in ONE kernel (mmb_mm2_stream_project): x, aux (and the column
    bounds) as mm2_stream, plus the MMB2 rows of mm2_project -- the sums s
    stay in LDS.  Returns (x, aux, mmb2)."""
    dev = audio.device
    if out is None:
        out = (torch.empty((n, d), dtype=torch.float32, device=dev),
               torch.empty((3, n), dtype=torch.float32, device=dev),
               torch.empty((n, d), dtype=torch.float32, device=dev))
    num, aux, mmb2 = out
    proj.enable_pieces()
    V = table.shape[0] if table is not None else 0
    _check_colmax_ws(colmax_ws, d)
    L.call("mmb_mm2_stream_project", L.ptr(ids32), L.ptr(table), V, L.ptr(wtab32),
           L.ptr(text_dense), L.ptr(w_dense), L.ptr(audio), L.ptr(visual), n, t, d, a, vd,
           L.ptr(proj.wpieces), L.ptr(proj.c0), L.ptr(num), L.ptr(aux), L.ptr(mmb2), L.ptr(flag),
           L.ptr(colmax), L.ptr(colmax_ws), L.stream_ptr())
    return num, aux, mmb2


def _check_colmax_ws(colmax_ws, d: int) -> None:
    """The C ABI takes the workspace as a bare pointer; the mirror checks its
    size (mmb_mm2_colmax_ws_bytes grew by 16 bytes in r05, include/mmb.h)."""
    if colmax_ws is None:
        return
    need = int(L.query("mmb_mm2_colmax_ws_bytes", d))
    have = colmax_ws.numel() * colmax_ws.element_size()
    if have < need:
        raise L.MMBError(f"colmax_ws holds {have} bytes; mmb_mm2_colmax_ws_bytes({d}) = {need}")


def s_buffer(n: int, kp: int, s_half: bool, device) -> torch.Tensor:
    if s_half:
        return torch.empty((n, 2 * kp), dtype=torch.float16, device=device)
    return torch.empty((n, kp), dtype=torch.float32, device=device)


def x3_supported(proj: "MMB2Projection") -> bool:
    """The x3 kernel's LDS chunk rings fit d < 320 (the D=300 configs)."""
    return proj.ldw <= 320


def project_split_ws(n: int, kp: int, device, slices: int = 0):
    """Scratch of the split-K projection (mmb_mm2_project_x3_split), or None
    where the rows alone fill the chip (one slice)."""
    if int(L.query("mmb_mm2_project_x3_split_slices", n, kp)) < 2 and slices < 2:
        return None
    nb = int(L.query("mmb_mm2_project_x3_split_ws_bytes", n, kp, slices))
    return torch.empty(max(nb, 16), dtype=torch.uint8, device=device)


def mm2_project(s, num, aux, proj: MMB2Projection, out=None, pc=None, sif_out=None, split=None,
                slices: int = 0):
    """fp16 s (s_half stream output): the fp16 hi/lo split MFMA GEMM
    (mmb_mm2_project_x3); fp32 s: the fp32-MFMA GEMM.  Same epilogue.
    With `pc` ([1, D] f64) and `sif_out` the x3 kernel also writes the
    PC-removed a2 rows (mmb_mm2_project_x3_rmpc, fp16 s only).  With `split`
    (project_split_ws) a few rows' K loop runs over several workgroups per
    row tile (mmb_mm2_project_x3_split, fp16 s)."""
    n = num.shape[0]
    if out is None:
        out = torch.empty((n, proj.d), dtype=torch.float32, device=num.device)
    if split is not None and s.dtype == torch.float16:
        L.call("mmb_mm2_project_x3_split", L.ptr(s), L.ptr(num), L.ptr(aux), L.ptr(proj.wsplit),
               proj.ldw, L.ptr(proj.c0), n, proj.kp, proj.d, L.ptr(out), L.ptr(pc),
               L.ptr(sif_out), int(slices), L.ptr(split), split.numel(), L.stream_ptr())
        return out
    if pc is not None:
        if s.dtype != torch.float16 or pc.shape[0] != 1 or sif_out is None:
            raise L.MMBError("fused PC removal needs fp16 s, npc = 1 and sif_out")
        L.call("mmb_mm2_project_x3_rmpc", L.ptr(s), L.ptr(num), L.ptr(aux), L.ptr(proj.wsplit),
               proj.ldw, L.ptr(proj.c0), n, proj.kp, proj.d, L.ptr(out), L.ptr(pc),
               L.ptr(sif_out), L.stream_ptr())
        return out
    if s.dtype == torch.float32:
        L.call("mmb_mm2_project", L.ptr(s), L.ptr(num), L.ptr(aux), L.ptr(proj.wm), proj.ldw,
               L.ptr(proj.c0), n, proj.kp, proj.d, L.ptr(out), L.stream_ptr())
    elif s.dtype == torch.float16:
        L.call("mmb_mm2_project_x3", L.ptr(s), L.ptr(num), L.ptr(aux), L.ptr(proj.wsplit),
               proj.ldw, L.ptr(proj.c0), n, proj.kp, proj.d, L.ptr(out), L.stream_ptr())
    else:
        raise L.MMBError(f"unsupported s dtype {s.dtype}")
    return out


class _NullSpan:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


class _EventSpan:
    """Records a timing event pair on the current stream around a block."""

    def __init__(self, sink: list):
        self.sink = sink

    def __enter__(self):
        self.a = torch.cuda.Event(enable_timing=True)
        self.a.record()
        return self

    def __exit__(self, *exc):
        b = torch.cuda.Event(enable_timing=True)
        b.record()
        self.sink.append((self.a, b))
        return False


def side_cu_set(n_cu: int, side: int, layout: str = "balanced") -> list[int]:
    """CU-mask bits for the side stream of the overlapped step.

    strided: evenly spaced bits; high: the top `side` bits; balanced: the same
    count in every block of 32 bits AND in every residue class mod 8, with the
    residues rotated from block to block -- even over the XCDs whether the
    driver deals mask bits to XCDs round-robin or in blocks of 32."""
    if layout == "strided":
        step = n_cu / side
        return sorted({int(i * step) for i in range(side)})
    if layout == "high":
        return list(range(n_cu - side, n_cu))
    if layout != "balanced":
        raise ValueError(f"unknown side CU layout {layout!r}")
    blocks = max(1, n_cu // 32)
    per = max(1, side // blocks)
    out = []
    for b in range(blocks):
        for j in range(per):
            out.append(32 * b + 8 * (j // 8) + (j + b * per) % 8)
    return sorted(set(c for c in out if c < n_cu))


# Splits below this many utterances take the exact f64 Gram (mmb_gram): at
# dataset sizes (MOSI 229-1284, POM 100-203 rows) it costs microseconds, and
# sklearn's transposed branch (n < d: a rank-n Gram) is where the int8 Gram's
# ~1e-10 relative error reached the PC at 2e-8 (r04d, real POM valid split);
# the int8 Gram pays from tens of thousands of rows up.
GRAM_I8_MIN_ROWS = 1 << 15

# Steps of at most this many rows fork the projection beside the Gram -> PC
# solve chain (FusedStep.fork): latency-bound kernels side by side.
FORK_PROJECTION_MAX_ROWS = 4096


class FusedStep:
    """One pass of the north-star hot path over a batch of utterances resident
    in HBM (bench 'step'): both the SIF text embedding (a1-a5, PC-removed) and
    the closed-form MMB2 embedding (a6-a8) of every utterance.

      mm2_stream   ids/table/wtab + audio + visual -> x, s, aux  (HBM-bound)
      gram         x -> G (fp64 MFMA)                  [+ RCCL all-reduce of G]
      pc_solve     G -> pc (1 workgroup)
      pc_remove    x, pc -> sif                          (HBM-bound)
      mm2_prepare  generator weights -> Wm, c0, fp16 hi/lo split
      mm2_project  s, x, aux, Wm -> mmb2 (fp16-split MFMA + fused normalisation;
                   the weighted text sum is x * count)

    With one chunk, npc = 1 and the fp16 split (the bench shape) the order is
    stream, Gram, PC solve, then ONE projection kernel that also writes the
    PC-removed rows (mmb_mm2_project_x3_rmpc): the removal re-reads x from
    cache instead of a separate HBM pass (`fuse_remove=False` keeps the
    separate pc_remove kernel).

    x is the a2 row (weighted text sum / count, the exact f32 division of
    sif_functions.py:55) written once by the stream kernel, so the Gram and
    the removal read it without dividing.

    With `chunks` > 1 the utterances are cut into row chunks (multiples of 256
    rows) and pipelined: chunk 0's stream kernel runs on every CU; then chunk
    c's stream kernel runs on the main stream while chunk c-1's projection and
    Gram partials (mmb_gram_part) run on a side stream; the last chunk's
    projection runs on every CU again, one mmb_gram_finish sums the partials,
    and the PC solve and removal follow.  `side_cus` > 0 puts the two streams
    on disjoint CU sets (CU-masked HIP streams; grid-stride kernels size their
    grids from the mask).  Measured on MI355X (1M utterances)
    the overlap does not pay: beside the MFMA-bound kernels the HBM-bound
    stream kernel slows by about what the projection hides (8 chunks, shared
    CUs / 64 balanced side CUs / 96 'high' side CUs: 28.5 / 30.7 / 28.8 ms per
    step against 28.6 ms unpipelined), so the default is one chunk.

    Small steps (the dataset splits, r06): `split_stream` cuts
    a few long rows over workgroups (mmb_mm2_stream_split), `split_projection`
    runs the projection split-K (mmb_mm2_project_x3_split; K summed in another
    f32 order than the one-pass kernel), and `fork_projection` runs it on a
    side stream beside Gram -> PC solve; each is chosen by shape when left at
    its default.
    """

    def __init__(self, inputs: dict, networks: dict, npc: int = 1, allreduce=None,
                 n_total: int | None = None, row0: int = 0, chunks: int | None = None,
                 side_cus: int = 0, side_layout: str = "balanced", fuse_remove: bool = True,
                 gram_kind: str | None = None, stream_project: bool | None = None,
                 narrow_fused: bool | None = None, check_each_run: bool = False,
                 fork_projection: bool | None = None, split_stream: bool | None = None,
                 split_projection: bool = True):
        self.inp = inputs
        self.check_each_run = check_each_run
        self.ids = inputs["ids"]
        self.n, self.t = self.ids.shape
        self.table = inputs["table"]
        self.V, self.d = self.table.shape
        self.a = inputs["audio"].shape[-1]
        self.vd = inputs["visual"].shape[-1]
        dev = self.table.device
        self.proj = MMB2Projection(networks, self.d, self.a, self.vd, self.t, dev)
        kp = self.proj.kp
        self.x = torch.empty((self.n, self.d), dtype=torch.float32, device=dev)
        self.s_half = x3_supported(self.proj)
        # stream + projection in one kernel (s never in HBM): one chunk, the
        # shapes the kernel takes, and wide frames (fused_pays);
        # MMB_STREAM_PROJECT=0 / 1 forces the two kernels / the fused one
        if stream_project is None:
            env = os.environ.get("MMB_STREAM_PROJECT")
            stream_project = fused_pays(self.a, self.vd) if env is None else env != "0"
        self.stream_project = (bool(stream_project) and (chunks or 1) == 1 and self.s_half
                               and stream_project_supported(self.t, self.d, self.a, self.vd))
        # narrow frame widths (MOSI): stream and projection in ONE kernel with
        # the per-word text cache (mmb_mm2_stream_project_narrow), one chunk;
        # MMB_NARROW_FUSED=0 / 1 forces the two kernels / the fused one
        if narrow_fused is None:
            env = os.environ.get("MMB_NARROW_FUSED")
            narrow_fused = True if env is None else env != "0"
        self.narrow_fused = (bool(narrow_fused) and not self.stream_project and (chunks or 1) == 1
                             and self.s_half
                             and narrow_fused_supported(self.t, self.d, self.a, self.vd, self.V))
        self.s = (None if (self.stream_project or self.narrow_fused)
                  else s_buffer(self.n, kp, self.s_half, dev))
        if self.stream_project:
            self.proj.enable_pieces()
        if self.narrow_fused:
            self.proj.enable_text_cache(self.table, inputs["wtab"])
        self.G = torch.empty((self.d, self.d), dtype=torch.float64, device=dev)
        self.pc_buf = torch.empty((npc, self.d), dtype=torch.float64, device=dev)
        self.solve_ws = (torch.zeros(L.query("mmb_pc_solve_mc_ws_bytes", self.d), dtype=torch.uint8,
                                     device=dev) if self.d <= PC_SOLVE_MC_MAX_D else None)
        self.sif = torch.empty((self.n, self.d), dtype=torch.float32, device=dev)
        self.mmb2 = torch.empty((self.n, self.d), dtype=torch.float32, device=dev)
        check_npc(npc)
        self.npc = npc
        self.allreduce = allreduce
        self.n_total = self.n if n_total is None else n_total
        self.row0 = row0
        self.flag = torch.zeros(1, dtype=torch.int32, device=dev)
        if chunks is None:
            chunks = 1
        if self.n_total < self.d:  # sklearn's transposed branch needs X^T Omega of all rows
            chunks = 1
        chunks = max(1, min(chunks, self.n))
        step = -(-self.n // chunks)
        step = -(-step // 256) * 256  # 16-byte aligned chunk starts (two-phase Gram)
        self.bounds = [(r, min(r + step, self.n)) for r in range(0, self.n, step)] or [(0, 0)]
        self.step_rows = step
        # aux is planar per chunk: chunk [r0, r1) owns flat[3 r0 : 3 r1] as [3][r1 - r0]
        self.aux_flat = torch.empty((3 * self.n,), dtype=torch.float32, device=dev)
        self.gram_parts = len(self.bounds) > 1 and self.d % 4 == 0 and self.d <= 320
        self.fused_remove = (fuse_remove and len(self.bounds) == 1 and npc == 1 and self.s_half
                             and not self.narrow_fused)
        # Gram of the one-chunk step: "i8" (mmb_gram_i8, int8 digits of the
        # column-bounded fixed-point x, ~1e-10 of exact; the bounds come from
        # the stream kernel) or "f64" (mmb_gram, exact f64 products).
        # MMB_GRAM overrides the default (A/B runs).
        if gram_kind is None:
            gram_kind = os.environ.get("MMB_GRAM", "i8" if self.n_total >= GRAM_I8_MIN_ROWS
                                       else "f64")
        if gram_kind not in ("i8", "f64"):
            raise ValueError(f"gram_kind must be 'i8' or 'f64', not {gram_kind!r}")
        self.gram_i8 = (gram_kind == "i8" and len(self.bounds) == 1 and self.d % 4 == 0
                        and self.d <= 304)
        if self.gram_i8:
            self.colmax = torch.zeros((self.d,), dtype=torch.int32, device=dev)
            nb = L.query("mmb_mm2_colmax_ws_bytes", self.d)
            self.colmax_ws = torch.empty((nb + 15) // 16 * 16, dtype=torch.uint8, device=dev)
        else:
            self.colmax = self.colmax_ws = None
        # a few long rows (POM's splits): every utterance's tokens and each
        # modality's frames on workgroups of their own (mmb_mm2_stream_split),
        # so 100-203 rows fill the chip instead of one workgroup each
        self.split = None
        if split_stream is None:
            split_stream = True
        if (split_stream and not self.stream_project and not self.narrow_fused
                and len(self.bounds) == 1
                and self.t > 64 and 0 < self.n <= L.cu_count(dev)):
            self.split = split_ws(self.n, self.t, self.d, self.a, self.vd, dev)
        # small steps (the dataset splits): the projection runs on a forked
        # stream beside the Gram -> PC solve chain, and the removal is its own
        # small launch, instead of the projection waiting for the PC to fuse
        # the removal into its tail (that saves an HBM pass only at scale)
        if fork_projection is None:
            fork_projection = self.n <= FORK_PROJECTION_MAX_ROWS
        self.fork = torch.cuda.Stream(device=dev) if self.fused_remove and fork_projection else None
        # a few rows: the projection's K loop split over workgroups
        self.proj_split = (project_split_ws(self.n, kp, dev)
                           if split_projection and self.s is not None and self.s_half
                           and len(self.bounds) == 1 else None)
        self.gws = GramWorkspace(max(r1 - r0 for r0, r1 in self.bounds), self.d, dev)
        self.side = torch.cuda.Stream(device=dev) if len(self.bounds) > 1 else None
        self.main = None
        self._cu_streams = []
        self._events = [torch.cuda.Event() for _ in self.bounds]
        if side_cus and self.side is not None:
            # disjoint CU sets: the stream kernel on `main`, the projection +
            # Gram of the previous chunk on `side`
            n_cu = L.cu_count(dev)
            side_set = side_cu_set(n_cu, side_cus, side_layout)
            main_set = [c for c in range(n_cu) if c not in set(side_set)]
            self._cu_streams = [L.CUStream(main_set, dev), L.CUStream(side_set, dev)]
            self.main, self.side = self._cu_streams[0].torch, self._cu_streams[1].torch

    def check(self):
        """Raise what the reference would have raised for the last step(s):
        IndexError for a token id >= V, ValueError for an utterance whose SIF
        weights are all 0 (the PC step of the split is then undefined),
        RuntimeError if the fused kernel's hand-over timed out.  Reads the flag
        word (one device sync); the flag accumulates until `reset()`.

        Sharded (an `allreduce` given), the three flag bits are summed over
        the ranks first -- one small all-reduce, only here -- so EVERY rank
        raises the same error for a bad utterance on any rank (a rank that
        raised alone would leave the others waiting in the next step's Gram
        all-reduce).  A NaN row reaches every rank's PC through the Gram anyway
        (check_pc_finite)."""
        flag = self.flag
        if self.allreduce is not None:
            bits = (L.MMB_FLAG_ID_RANGE, L.MMB_FLAG_ZERO_WEIGHTS, L.MMB_FLAG_SYNC_TIMEOUT)
            t = torch.stack([(flag[0] & b) != 0 for b in bits]).to(torch.int32)
            self.allreduce(t)
            flag = sum((t[i] > 0).to(torch.int32) * b for i, b in enumerate(bits)).reshape(1)
        self.raise_status(int(self.status(flag).item()))  # the one device sync

    def status(self, flag=None, out=None) -> torch.Tensor:
        """[1] int32 on the device: the flag bits | PC_NONFINITE when the last
        step's PC is not finite -- what check() reads back, formed without a
        sync (StepGraph captures it into the graph)."""
        flag = self.flag if flag is None else flag
        pc = getattr(self, "pc", None)
        if pc is None:
            return torch.add(flag, 0, out=out)
        if out is None:
            out = torch.empty(1, dtype=torch.int32, device=flag.device)
        # one launch (mmb_step_status): eight elementwise torch kernels here
        # were ~40 us of every dataset split's graph (r06 kernel trace)
        L.call("mmb_step_status", L.ptr(flag), L.ptr(pc), pc.numel(), PC_NONFINITE, L.ptr(out),
               L.stream_ptr())
        return out

    def raise_status(self, v: int):
        """check()'s verdict on a status word read back (status())."""
        if self.solve_ws is not None and v & (L.MMB_FLAG_SYNC_TIMEOUT | PC_NONFINITE):
            # an aborted solve leaves its control words set (and a NaN PC):
            # hand the next launch a zeroed workspace again
            self.solve_ws[:16].zero_()
        check_flag_bits(v & (PC_NONFINITE - 1), self.V, zero_weights=True)
        if v & PC_NONFINITE:
            raise ValueError("Input X contains NaN or infinity: the split's Gram is not finite "
                             "(an all-zero-weight utterance on some rank, or non-finite inputs), "
                             "which the reference's TruncatedSVD rejects (sif_functions.py:65-67)")

    def reset(self):
        self.flag.zero_()

    def aux_of(self, c: int) -> torch.Tensor:
        r0, r1 = self.bounds[c]
        return self.aux_flat[3 * r0:3 * r1].view(3, r1 - r0)

    @property
    def aux(self) -> torch.Tensor:
        """[3, N] planar aux (count, total weight, row scale) of a one-chunk step."""
        if len(self.bounds) != 1:
            raise ValueError("aux is planar per chunk when chunks > 1; use aux_of(c)")
        return self.aux_of(0)

    def _stream_chunk(self, c: int):
        r0, r1 = self.bounds[c]
        inp = self.inp
        mm2_stream(r1 - r0, self.t, self.d, self.a, self.vd, inp["audio"][r0:r1],
                   inp["visual"][r0:r1], ids32=self.ids[r0:r1], table=self.table,
                   wtab32=inp["wtab"], flag=self.flag, s_half=self.s_half,
                   out=(self.x[r0:r1], self.s[r0:r1], self.aux_of(c)),
                   colmax=self.colmax, colmax_ws=self.colmax_ws, split=self.split)

    def _consume_chunk(self, c: int):
        r0, r1 = self.bounds[c]
        aux = self.aux_of(c)
        mm2_project(self.s[r0:r1], self.x[r0:r1], aux, self.proj, out=self.mmb2[r0:r1],
                    split=self.proj_split)  # (None past one chunk)
        if self.gram_parts:
            L.call("mmb_gram_part", L.ptr(self.x[r0:r1]), None, r1 - r0,
                   self.step_rows, self.d, int(c > 0), L.ptr(self.gws.buf), L.stream_ptr())
        elif self.gram_i8:  # one chunk
            gram_i8(self.x, self.colmax, self.G, ws=self.gws)
        else:
            gram(self.x[r0:r1], None, self.G, accumulate=c > 0, ws=self.gws)

    def _solve(self, trace, mark):
        """G (this rank's rows) -> pc: Omega, RCCL all-reduce of G, the solve."""
        d, k = self.d, self.npc + N_OVERSAMPLES
        if (self.n_total < d and self.allreduce is None and self.solve_ws is not None
                and k <= 16):
            # the transposed branch, unsharded: X^T Omega and the squared
            # matrix in one launch in front of the solve (mmb_pc_solve_mc_xt)
            om = omega(self.n_total, k, self.table.device)
            with mark("pc_solve"):
                L.call("mmb_pc_solve_mc_xt", L.ptr(self.G), d, L.ptr(self.x), self.n, L.ptr(om), k,
                       self.npc, N_ITER, L.ptr(self.pc_buf), L.ptr(self.solve_ws), L.ptr(self.flag),
                       L.stream_ptr())
            return self.pc_buf
        with mark("pc_start"):
            if self.n_total >= d:
                z0, transposed = omega(d, k, self.table.device), False
            else:
                om = omega(self.n_total, k, self.table.device)[self.row0:self.row0 + self.n]
                z0, transposed = xt_omega(self.x, None, om.contiguous()), True
        if self.allreduce is not None:
            with mark("allreduce"):
                self.allreduce(self.G)
                if transposed:
                    self.allreduce(z0)
        with mark("pc_solve"):
            return pc_solve(self.G, z0, self.npc, transposed, out=self.pc_buf, flag=self.flag,
                            ws=self.solve_ws)

    def run(self, trace: dict | None = None, check: bool | None = None):
        """One step.  With `trace` (a dict), HIP events are recorded on the
        stream each phase runs on: trace[phase] gets (start, end) pairs.
        With `check` (default: the constructor's `check_each_run`) the step
        ends with check() -- one device sync -- and raises like the
        reference; without it the step never synchronises and the caller
        calls check() when it wants the verdict (bench.py: once, after the
        timed steps)."""
        out = self._run(trace)
        if self.check_each_run if check is None else check:
            self.check()
        return out

    def _run(self, trace, fork: bool = True):
        def mark(name):
            if trace is None:
                return _NullSpan()
            return _EventSpan(trace.setdefault(name, []))

        d, k = self.d, self.npc + N_OVERSAMPLES
        nb = len(self.bounds)
        with mark("mm2_prepare"):
            self.proj.refresh_if_changed()
        if self.narrow_fused:
            inp = self.inp
            with mark("mm2_stream_project_narrow"):
                mm2_stream_project_narrow(self.n, self.t, self.d, self.a, self.vd, inp["audio"],
                                          inp["visual"], self.proj, self.ids, self.table,
                                          inp["wtab"], flag=self.flag,
                                          out=(self.x, self.aux_of(0), self.mmb2),
                                          colmax=self.colmax, colmax_ws=self.colmax_ws)
            with mark("gram"):
                if self.gram_i8:
                    gram_i8(self.x, self.colmax, self.G, ws=self.gws)
                else:
                    gram(self.x, None, self.G, ws=self.gws)
            pc = self._solve(trace, mark)
            with mark("pc_remove"):
                remove_pc(self.x, None, pc, out=self.sif)
            self.pc = pc
            return self.sif, self.mmb2
        if self.stream_project:
            inp = self.inp
            with mark("mm2_stream_project"):
                mm2_stream_project(self.n, self.t, self.d, self.a, self.vd, inp["audio"],
                                   inp["visual"], self.proj, ids32=self.ids, table=self.table,
                                   wtab32=inp["wtab"], flag=self.flag,
                                   out=(self.x, self.aux_of(0), self.mmb2), colmax=self.colmax,
                                   colmax_ws=self.colmax_ws)
            with mark("gram"):
                if self.gram_i8:
                    gram_i8(self.x, self.colmax, self.G, ws=self.gws)
                else:
                    gram(self.x, None, self.G, ws=self.gws)
            pc = self._solve(trace, mark)
            with mark("pc_remove"):
                remove_pc(self.x, None, pc, out=self.sif)
            self.pc = pc
            return self.sif, self.mmb2
        with mark("mm2_stream"):
            self._stream_chunk(0)  # every CU
        if self.fork is not None:
            # the projection beside the Gram -> solve chain; with fork=False
            # (inside a concurrent StepGraph) the same kernels in one stream,
            # so the rows are the forked step's bit for bit
            caller = torch.cuda.current_stream(self.table.device)
            side = self.fork if fork else caller
            if fork:
                side.wait_stream(caller)
            with torch.cuda.stream(side):
                with mark("mm2_project"):
                    mm2_project(self.s, self.x, self.aux_of(0), self.proj, out=self.mmb2,
                                split=self.proj_split)
            with mark("gram"):
                if self.gram_i8:
                    gram_i8(self.x, self.colmax, self.G, ws=self.gws)
                else:
                    gram(self.x, None, self.G, ws=self.gws)
            pc = self._solve(trace, mark)
            with mark("pc_remove"):
                remove_pc(self.x, None, pc, out=self.sif)
            if fork:
                caller.wait_stream(side)
            self.pc = pc
            return self.sif, self.mmb2
        if self.fused_remove:
            with mark("gram"):
                if self.gram_i8:
                    gram_i8(self.x, self.colmax, self.G, ws=self.gws)
                else:
                    gram(self.x, None, self.G, ws=self.gws)
            pc = self._solve(trace, mark)
            with mark("mm2_project+pc_remove"):
                mm2_project(self.s, self.x, self.aux_of(0), self.proj, out=self.mmb2, pc=pc,
                            sif_out=self.sif, split=self.proj_split)
            self.pc = pc
            return self.sif, self.mmb2
        if nb > 1:
            caller = torch.cuda.current_stream(self.table.device)
            main = self.main if self.main is not None else caller
            side = self.side
            ev = self._events
            ev[0].record(caller)
            if main is not caller:
                main.wait_stream(caller)
            side.wait_stream(caller)
            for c in range(1, nb):
                with torch.cuda.stream(main):
                    with mark("mm2_stream"):
                        self._stream_chunk(c)
                    if c < nb - 1:
                        ev[c].record(main)
                with torch.cuda.stream(side):
                    side.wait_event(ev[c - 1])
                    with mark("mm2_project+gram"):
                        self._consume_chunk(c - 1)
            if main is not caller:
                caller.wait_stream(main)
            caller.wait_stream(side)
        with mark("mm2_project+gram"):
            self._consume_chunk(nb - 1)  # every CU
        if self.gram_parts:
            with mark("gram_finish"):
                L.call("mmb_gram_finish", self.step_rows, d, L.ptr(self.G), 0, L.ptr(self.gws.buf),
                       L.stream_ptr())
        pc = self._solve(trace, mark)
        with mark("pc_remove"):
            for c, (r0, r1) in enumerate(self.bounds):
                remove_pc(self.x[r0:r1], None, pc, out=self.sif[r0:r1])
        self.pc = pc
        return self.sif, self.mmb2


class StepGraph:
    """One or more FusedSteps' device work captured ONCE as a HIP graph and
    replayed: the per-split call pattern of the reference (SIF once per split,
    each split with its own PC: simplesif.py:296-311) pays the host launch
    cost of ~10 kernels per split on every call; a replay is one launch.

    `concurrent=True` captures every step on its own stream (fork / join
    branches of the graph), so independent splits overlap on the chip -- the
    PC solves of different splits (each ceil(d/16) workgroups) run side by
    side instead of back to back.  Steps are warmed up eagerly first (weight
    merge, Omega upload, workspaces); a later in-place update of a generator
    parameter is re-merged eagerly before the replay (the merge writes the
    buffers the graph reads).  No host sync unless `check`."""

    def __init__(self, steps, concurrent: bool = False, warmup: int = 1):
        self.steps = list(steps) if isinstance(steps, (list, tuple)) else [steps]
        dev = self.steps[0].table.device
        caller = torch.cuda.current_stream(dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(caller)
        with torch.cuda.stream(side):
            for _ in range(warmup):
                for st in self.steps:
                    st.run()
        caller.wait_stream(side)
        torch.cuda.synchronize(dev)
        for st in self.steps:
            # the warm-up's verdict first: a flag (or an aborted solve's NaN
            # PC) raises here instead of being cleared by reset() and leaving
            # every replay to run on a dirty workspace
            st.check()
            st.reset()
        self._branches = ([torch.cuda.Stream(device=dev) for _ in self.steps]
                          if concurrent and len(self.steps) > 1 else None)
        # every step's status word (FusedStep.status) is formed inside the
        # graph, so a checked replay reads ONE small tensor back (one sync for
        # all steps; check() per step took up to four)
        self._status = torch.zeros(len(self.steps), dtype=torch.int32, device=dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            cap = torch.cuda.current_stream(dev)
            if self._branches is None:
                self.outs = [st._run(None) for st in self.steps]
            else:
                self.outs = []
                # the steps run WITHOUT their forked projection here: the
                # splits' branches already overlap, and with the forks the
                # replay ran the branches one after the other (POM's two
                # splits 0.505 ms concurrent vs 0.503 serial; without 0.436,
                # r06 tools/pom_graph_ab.py); a fork joined back to its
                # branch stream also segfaulted the capture
                # (tools/dbg/fork_graph_probe.py)
                for st, br in zip(self.steps, self._branches):
                    br.wait_stream(cap)
                    with torch.cuda.stream(br):
                        self.outs.append(st._run(None, fork=False))
                for br in self._branches:
                    cap.wait_stream(br)
            for i, st in enumerate(self.steps):
                if st.allreduce is None:
                    st.status(out=self._status[i:i + 1])

    def run(self, check: bool = False):
        for st in self.steps:
            st.proj.refresh_if_changed()
        self.graph.replay()
        if check:
            words = self._status.tolist()  # the one sync
            for st, v in zip(self.steps, words):
                if st.allreduce is not None:
                    st.check()  # (its flag bits cross ranks: check()'s all-reduce)
                else:
                    st.raise_status(v)
        return self.outs if len(self.steps) > 1 else self.outs[0]
