"""ctypes binding of libmmb.so (the C ABI declared in include/mmb.h).

torch is imported first on purpose: torch ships its own HIP runtime with the
same soname (libamdhip64.so.7) as /opt/rocm's, so loading libmmb.so after
torch makes it bind to the runtime torch already initialised — one HIP
runtime per process, and torch-allocated device pointers / torch streams are
valid inside libmmb.

There is no fallback: if libmmb.so is missing or no GPU is visible, every
entry point raises.  (Build it with `python -c "import __graft_entry__ as g;
g.build()"` or `make -C multimodal-baselines_amd/csrc`.)
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the dlopen below)

HERE = os.path.dirname(os.path.abspath(__file__))
# The product library.  No environment variable redirects it: the tools build
# (libmmb_diag.so, timing-only variants that write wrong rows by design) is
# loaded only by an explicit load(path) from tools/ or tests/variant_checks.py.
LIB_PATH = os.path.join(HERE, "libmmb.so")

MMB_FLAG_ID_RANGE = 1
MMB_FLAG_ZERO_WEIGHTS = 2
MMB_FLAG_SYNC_TIMEOUT = 4

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_F = ctypes.c_float
_S = ctypes.c_size_t

# name -> (restype, argtypes)
SIGNATURES = {
    "mmb_version": (_I, []),
    "mmb_seq2weight": (_I, [_P, _P, _L, _L, _P, _L, _P, _P, _P]),
    "mmb_sif_wavg": (_I, [_P, _L, _I, _P, _L, _I, _P, _P, _P, _P, _P, _P, _P]),
    "mmb_gram_workspace_bytes": (_S, [_L, _I]),
    "mmb_gram": (_I, [_P, _P, _L, _I, _P, _I, _P, _P]),
    "mmb_gram_part": (_I, [_P, _P, _L, _L, _I, _I, _P, _P]),
    "mmb_colmax": (_I, [_P, _L, _I, _P, _I, _P]),
    "mmb_gram_i8": (_I, [_P, _P, _L, _I, _P, _I, _P, _P]),
    "mmb_gram_finish": (_I, [_L, _I, _P, _I, _P, _P]),
    "mmb_xt_omega": (_I, [_P, _P, _L, _I, _P, _I, _P, _P]),
    "mmb_pc_solve": (_I, [_P, _I, _P, _I, _I, _I, _I, _P, _P]),
    "mmb_pc_solve_mc_ws_bytes": (_S, [_I]),
    "mmb_step_status": (_I, [_P, _P, _I, _I, _P, _P]),
    "mmb_pc_solve_mc_xt": (_I, [_P, _I, _P, _L, _P, _I, _I, _I, _P, _P, _P, _P]),
    "mmb_pc_solve_mc": (_I, [_P, _I, _P, _I, _I, _I, _I, _P, _P, _P, _P]),
    "mmb_pc_remove": (_I, [_P, _P, _L, _I, _P, _I, _P, _P, _P]),
    "mmb_gram_f64": (_I, [_P, _L, _I, _P, _I, _P, _P]),
    "mmb_xt_omega_f64": (_I, [_P, _L, _I, _P, _I, _P, _P]),
    "mmb_pc_remove_f64": (_I, [_P, _L, _I, _P, _I, _P, _P]),
    "mmb_host_randn": (_I, [ctypes.c_uint32, _L, _P]),
    "mmb_cu_count": (_I, [_I, _P]),
    "mmb_stream_create_cu_mask": (_I, [_P, _I, _P]),
    "mmb_stream_destroy": (_I, [_P]),
    "mmb_probe_copy": (_I, [_P, _P, _L, _I, _I, _P]),
    "mmb_probe_read": (_I, [_P, _L, _I, _I, _P, _P]),
    "mmb_calc_weights": (_I, [_P, _L, _I, _P, _P, _P, _P, _P]),
    "mmb_mm2_k": (_I, [_I, _I, _I]),
    "mmb_mm2_ldw": (_I, [_I]),
    "mmb_mm2_stream": (_I, [_P, _P, _L, _P, _P, _P, _P, _P, _P, _L, _I, _I, _I, _I, _P, _P, _I,
                            _P, _P, _P, _P, _P]),
    "mmb_mm2_colmax_ws_bytes": (_S, [_I]),
    "mmb_mm2_stream_split_parts": (_I, [_L, _I]),
    "mmb_mm2_stream_split_ws_bytes": (_S, [_L, _I, _I, _I, _I, _I]),
    "mmb_mm2_stream_split": (_I, [_P, _P, _L, _P, _P, _P, _P, _P, _P, _L, _I, _I, _I, _I, _P, _P,
                                  _I, _P, _P, _P, _P, _I, _P, _S, _P]),
    "mmb_mm2_stream_project_supported": (_I, [_I, _I, _I, _I]),
    "mmb_mm2_stream_project": (_I, [_P, _P, _L, _P, _P, _P, _P, _P, _L, _I, _I, _I, _I, _P, _P,
                                    _P, _P, _P, _P, _P, _P, _P]),
    "mmb_mm2_prepare": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _P, _I, _P, _P, _P]),
    "mmb_mm2_text_cache_bytes": (_S, [_L, _I]),
    "mmb_mm2_text_cache": (_I, [_P, _L, _I, _P, _P, _I, _P, _P]),
    "mmb_mm2_stream_project_narrow_supported": (_I, [_I, _I, _I, _I, _L]),
    "mmb_mm2_stream_project_narrow": (_I, [_P, _P, _L, _P, _P, _P, _P, _L, _I, _I, _I, _I, _P,
                                           _P, _P, _P, _P, _P, _P, _P, _P]),
    "mmb_mm2_split_bytes": (_S, [_I, _I, _I]),
    "mmb_mm2_split_pieces_bytes": (_S, [_I, _I, _I]),
    "mmb_mm2_split_pieces": (_I, [_P, _I, _I, _I, _I, _P, _P]),
    "mmb_mm2_project": (_I, [_P, _P, _P, _P, _I, _P, _L, _I, _I, _P, _P]),
    "mmb_mm2_project_x3": (_I, [_P, _P, _P, _P, _I, _P, _L, _I, _I, _P, _P]),
    "mmb_mm2_project_x3_rmpc": (_I, [_P, _P, _P, _P, _I, _P, _L, _I, _I, _P, _P, _P, _P]),
    "mmb_mm2_project_x3_split_slices": (_I, [_L, _I]),
    "mmb_mm2_project_x3_split_ws_bytes": (_S, [_L, _I, _I]),
    "mmb_mm2_project_x3_split": (_I, [_P, _P, _P, _P, _I, _P, _L, _I, _I, _P, _P, _P, _I, _P, _S,
                                      _P]),
    "mmb_mlp_forward": (_I, [_P, _P, _L, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "mmb_mlp_eval": (_I, [_P, _P, _P, _L, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "mmb_mlp_forward_train": (_I, [_P, _L, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "mmb_mlp_backward": (_I, [_P, _P, _L, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "mmb_mlp_workspace_bytes": (_S, [_I, _I]),
    "mmb_mlp_train": (_I, [_P, _P, _P, _L, _I, _I, _I, _I, _I, _F, _P, _P, _P, _P, _P,
                           _P, _P, _P, _L, _I, _I, _P, _P, _P, _P]),
    "mmb_word_pad": (_I, [_I]),
    "mmb_word_normalize": (_I, [_P, _L, _I, _P, _P]),
    "mmb_word_workspace_bytes": (_S, [_L, _I, _L]),
    "mmb_word_logprob_forward": (_I, [_P, _L, _I, _P, _L, _P, _P, _P, _I, _P, _P, _F, _I, _P, _P,
                                      _P, _P, _P, _P]),
    "mmb_word_logprob_backward": (_I, [_P, _L, _I, _L, _P, _P, _P, _I, _P, _P, _F, _P, _P, _P, _P,
                                       _P, _P]),
    "mmb_gauss_stats": (_I, [_P, _P, _L, _I, _I, _P, _P]),
    "mmb_gauss_loglik": (_I, [_P, _P, _P, _L, _I, _P, _P, _P, _P, _P]),
    "mmb_gauss_backward": (_I, [_P, _P, _P, _L, _I, _P, _P, _P, _P, _P, _P, _P]),
    "mmb_gauss_loglik_strided": (_I, [_P, _P, _P, _L, _I, _P, _P, _P, _P, _P, _P, _P]),
    "mmb_gauss_backward_strided": (_I, [_P, _P, _P, _L, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "mmb_layer_norm_backward": (_I, [_P, _P, _P, _P, _P, _L, _I, _P, _P, _P, _P]),
}

_lib = None


class MMBError(RuntimeError):
    pass


_loaded_path = None


def load(path=None):
    """dlopen the library once (no GPU needed to load or query symbols).

    `path` (tools only) names another build, e.g. the tools build
    libmmb_diag.so; it must be given before anything else loads the library,
    and a second, different path raises instead of silently mixing builds."""
    global _lib, _loaded_path
    want = os.path.abspath(path) if path is not None else None
    if _lib is not None:
        if want is not None and want != _loaded_path:
            raise MMBError(f"libmmb already loaded from {_loaded_path}; cannot switch to {want}")
        return _lib
    lib_path = want or LIB_PATH
    if _lib is None:
        if not os.path.exists(lib_path):
            raise ImportError(f"libmmb not built at {lib_path}; run `make -C "
                              f"{os.path.join(HERE, 'csrc')}` or __graft_entry__.build()")
        lib = ctypes.CDLL(lib_path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        _loaded_path = lib_path
    return _lib


def loaded_path():
    return _loaded_path


def call(name, *args):
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise MMBError(f"{name} failed with code {rc}" + (" (invalid argument)" if rc < 0 else
                                                            " (hipError)"))
    return rc


def query(name, *args):
    return getattr(load(), name)(*args)


def require_gpu() -> torch.device:
    if not torch.cuda.is_available():
        raise MMBError("libmmb computes on an MI355X (gfx950) GPU and has no CPU fallback; "
                       "no GPU is visible")
    load()
    return torch.device("cuda", torch.cuda.current_device())


def ptr(t) -> int | None:
    if t is None:
        return None
    if not t.is_cuda:
        raise MMBError("libmmb entry points take device tensors")
    if not t.is_contiguous():
        raise MMBError("libmmb entry points take contiguous tensors")
    return t.data_ptr()


def stream_ptr(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def host_randn(seed: int, count: int):
    """numpy RandomState(seed).normal(size=count), from the C++ MT19937 in libmmb."""
    import numpy as np

    out = np.empty(count, dtype=np.float64)
    call("mmb_host_randn", seed, count, out.ctypes.data if count else None)
    return out


def cu_count(device=None) -> int:
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else device
    out = ctypes.c_int(0)
    call("mmb_cu_count", dev.index or 0, ctypes.addressof(out))
    return out.value


class CUStream:
    """A HIP stream restricted to the CUs in `cus` (libmmb
    mmb_stream_create_cu_mask), usable as a torch stream via `.torch`."""

    def __init__(self, cus, device):
        n = max(cus) + 1
        words = (ctypes.c_uint32 * ((n + 31) // 32))()
        for c in cus:
            words[c // 32] |= 1 << (c % 32)
        handle = ctypes.c_void_p(0)
        with torch.cuda.device(device):
            call("mmb_stream_create_cu_mask", ctypes.addressof(words), len(words),
                 ctypes.addressof(handle))
        self.handle = handle.value
        self.cus = list(cus)
        self.torch = torch.cuda.ExternalStream(self.handle, device=device)

    def close(self):
        if self.handle:
            torch.cuda.synchronize()
            call("mmb_stream_destroy", self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
