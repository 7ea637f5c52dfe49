"""CPU: the C-ABI library loads and exports every symbol include/mmb.h declares.

No compute calls here (no GPU in the build container) except the host-only
RNG helper, which is checked bit for bit against numpy's legacy RandomState.
"""
import os
import re
import subprocess

import numpy as np
import pytest

import mmb_lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mmb.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mmb_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared_functions()
    assert "mmb_sif_wavg" in names and "mmb_pc_solve" in names and "mmb_mlp_train" in names
    assert len(names) >= 19


def test_library_exports_every_declared_symbol():
    lib = mmb_lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), f"{name} declared in mmb.h but not exported"


def test_ctypes_signatures_cover_header():
    assert set(declared_functions()) == set(mmb_lib.SIGNATURES)


def test_exports_are_c_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", mmb_lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (mmb_\w+)", out))
    assert set(declared_functions()) <= exported  # unmangled extern "C"


def test_product_library_reads_no_knobs():
    """The product library carries only the default kernels: no getenv, no
    MMB_* knob string, no timing-only DIAG build (those live in the tools
    build libmmb_diag.so, `make diag`)."""
    path = os.path.join(ROOT, "multimodal-baselines_amd", "libmmb.so")
    blob = open(path, "rb").read()
    assert b"DIAG" not in blob
    assert re.search(rb"MMB_[A-Z_]{3,}", blob) is None
    undef = subprocess.run(["nm", "-D", "--undefined-only", path], capture_output=True, text=True,
                           check=True).stdout
    assert "getenv" not in undef


def test_product_sources_carry_no_tools_code():
    """The product kernel sources hold only what libmmb.so runs (r06): no
    environment reads and no MMB_DIAG blocks -- the tools build's variants,
    knobs and probes live in tools/diag/ and plug into named MMB_HOOK_*
    points whose product defaults are compiled here."""
    csrc = os.path.join(ROOT, "multimodal-baselines_amd", "csrc")
    srcs = [f for f in os.listdir(csrc) if f.endswith((".hip", ".h", ".cpp"))]
    assert "sif_kernels.hip" in srcs and "pc_kernels.hip" in srcs
    for f in srcs:
        text = open(os.path.join(csrc, f)).read()
        assert "getenv" not in text, f
        assert "MMB_DIAG" not in text, f
    # the tails the tools build includes exist; the product's target is empty
    for tail in ("sif_tail.inc", "pc_tail.inc", "mm2_tail.inc", "diag_hooks.h"):
        assert os.path.exists(os.path.join(ROOT, "tools", "diag", tail)), tail
    code = re.sub(r"//[^\n]*", "", open(os.path.join(csrc, "mmb_no_tools.h")).read())
    assert code.strip() == ""


def test_library_carries_gfx950_code_objects():
    data = open(mmb_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version_and_shape_helpers():
    assert mmb_lib.query("mmb_version") >= 100
    assert mmb_lib.query("mmb_mm2_k", 300, 300, 300) == 1824
    assert mmb_lib.query("mmb_mm2_k", 300, 76, 48) == 864
    assert mmb_lib.query("mmb_mm2_ldw", 300) == 320
    assert mmb_lib.query("mmb_gram_workspace_bytes", 1_000_000, 300) > 0
    # arrival counter + abort word, then 2 x 4 hidden tiles x 32 rows x 16 outputs of f32 shares
    assert mmb_lib.query("mmb_mlp_workspace_bytes", 300, 100) == 16 + 4 * 2 * 4 * 32 * 16


@pytest.mark.parametrize("seed,rows,k", [(0, 300, 11), (0, 64, 11), (0, 1, 12), (7, 1000, 3)])
def test_host_randn_matches_numpy_randomstate(seed, rows, k):
    got = mmb_lib.host_randn(seed, rows * k)
    ref = np.random.RandomState(seed).normal(size=(rows, k)).ravel()
    assert np.array_equal(got, ref)


def test_invalid_arguments_rejected_without_gpu():
    # argument validation happens before any launch
    with pytest.raises(mmb_lib.MMBError):
        mmb_lib.call("mmb_pc_solve", None, 300, None, 11, 1, 7, 0, None, None)
    with pytest.raises(mmb_lib.MMBError):
        mmb_lib.call("mmb_host_randn", 0, -1, None)


def test_environment_cannot_redirect_the_product_library(tmp_path):
    """MMB_LIB_PATH (the round-3 A/B hook) no longer exists: a fresh process
    with it set to the tools build still loads libmmb.so; the tools build is
    reachable only through an explicit mmb_lib.load(path)."""
    import sys
    diag = os.path.join(ROOT, "tools", "diag", "libmmb_diag.so")
    code = ("import sys; sys.path.insert(0, %r); import mmb_lib; mmb_lib.load(); "
            "print(mmb_lib.loaded_path())" % os.path.join(ROOT, "multimodal-baselines_amd"))
    env = {**os.environ, "MMB_LIB_PATH": diag, "MMB_TOOLS_LIB": diag}
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         check=True).stdout.strip().splitlines()[-1]
    assert out == os.path.join(ROOT, "multimodal-baselines_amd", "libmmb.so")
    src = open(os.path.join(ROOT, "multimodal-baselines_amd", "mmb_lib.py")).read()
    assert "os.environ" not in src and "getenv" not in src


def test_second_library_path_is_refused():
    lib = mmb_lib.load()
    assert mmb_lib.load() is lib
    with pytest.raises(mmb_lib.MMBError):
        mmb_lib.load(os.path.join(ROOT, "tools", "diag", "libmmb_diag.so"))
