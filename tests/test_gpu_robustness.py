"""Robustness of the in-launch hand-overs and of captured steps, through the
PRODUCT library (no tools build needed).

The multi-workgroup PC solve (mmb_pc_solve_mc) and the regressor's training
launch (mmb_mlp_train) exchange tiles between workgroups through an arrival
counter and an abort word in a caller-owned workspace; the contract
(include/mmb.h) is that the caller hands the words over zeroed and a completed
launch leaves them zero.  These tests hand them over DIRTY -- an abort word
left set by an earlier aborted launch, a counter left at a stale count --
which is what the round-4 replay failure looked like, and check the whole
recovery path: the launch ends, flags MMB_FLAG_SYNC_TIMEOUT, writes a NaN PC
rather than a stale or half-exchanged one, the Python layer raises
RuntimeError and re-zeroes the words, and the next launch reproduces the clean
result bit for bit.  (The timeout itself -- a wait that runs out -- needs the
tools build's shortened wait budget: tests/test_gpu_variants.py.)

Also here: graph replays of the >= 32k-row steps (the int8-Gram path: column
bounds written by the stream kernel, reduced, then the Gram) on inputs that
change between replays, against an eager step; the narrow fused kernel's text
cache following a NEW weight tensor; and RCCL (backend "nccl") on the step's
path at world size 1.
Reference: /root/reference/sif_functions.py:58-67 (the PC the solve
replays), /root/reference/sentiment_model.py:52-265 (the training loop),
/root/reference/simplesif.py:296-311 (the per-split call pattern).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

import mmb_lib as L
import models
import pipeline as P
import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

# the two control words at the head of the solve / train workspaces
CTR, ABORT = 0, 1
DIRTY = [("abort word", ABORT, 1), ("stale count < T", CTR, 5), ("stale count >> T", CTR, 1000)]


def _gram(dev, n=2000, d=300, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(n, d, generator=g, device=dev, dtype=torch.float64) * 0.4
    x += 0.3 * torch.randn(d, generator=g, device=dev, dtype=torch.float64)
    return x.T @ x


def _set_word(ws: torch.Tensor, word: int, value: int):
    ws[:16].view(torch.int32)[word] = value


@pytest.mark.parametrize("what,word,value", DIRTY, ids=[d[0] for d in DIRTY])
def test_pc_solve_dirty_workspace_aborts_and_recovers(gpu, what, word, value):
    G = _gram(gpu)
    z0 = P.omega(300, 11, gpu)
    ws = torch.zeros(L.query("mmb_pc_solve_mc_ws_bytes", 300), dtype=torch.uint8, device=gpu)
    flag = torch.zeros(1, dtype=torch.int32, device=gpu)
    pc0 = P.pc_solve(G, z0, 1, False, flag=flag, ws=ws).clone()
    torch.cuda.synchronize()
    assert int(flag.item()) == 0 and not bool(ws[:16].any())  # a completed solve leaves ws zero

    _set_word(ws, word, value)
    pc = P.pc_solve(G, z0, 1, False, flag=flag, ws=ws)
    torch.cuda.synchronize()
    assert int(flag.item()) & L.MMB_FLAG_SYNC_TIMEOUT, what
    assert bool(torch.isnan(pc).all()), what  # never a stale or half-exchanged PC
    # without a caller flag, pc_solve checks its own, raises and re-zeroes
    with pytest.raises(RuntimeError, match="timed out"):
        P.pc_solve(G, z0, 1, False, ws=ws)
    assert not bool(ws[:16].any())
    flag.zero_()
    pc1 = P.pc_solve(G, z0, 1, False, flag=flag, ws=ws)
    torch.cuda.synchronize()
    assert int(flag.item()) == 0 and torch.equal(pc0, pc1)


def _bench_like_step(dev, n, mosi, seed=91):
    A, Vd, V, T = (76, 48, 3016, 20) if mosi else (300, 300, 50_000, 40)
    inp = synth.device_workload(n, T, V, A=A, Vd=Vd, seed=seed, device=dev)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(dev)
    return inp, gen


@pytest.mark.parametrize("what,word,value", DIRTY, ids=[d[0] for d in DIRTY])
def test_fused_step_dirty_solve_workspace_raises_then_recovers(gpu, what, word, value):
    """FusedStep.check() raises RuntimeError on an aborted solve (flag bit,
    NaN PC), re-zeroes the workspace, and the next checked run equals the
    clean one bit for bit."""
    inp, gen = _bench_like_step(gpu, 40_000, mosi=True)
    st = P.FusedStep(inp, gen.networks())
    assert st.narrow_fused and st.gram_i8
    s0, m0 = [t.clone() for t in st.run(check=True)]
    pc0 = st.pc.clone()
    _set_word(st.solve_ws, word, value)
    st.run()
    with pytest.raises(RuntimeError, match="timed out"):
        st.check()
    assert not bool(st.solve_ws[:16].any())
    st.reset()
    s1, m1 = st.run(check=True)
    assert torch.equal(s0, s1) and torch.equal(m0, m1) and torch.equal(pc0, st.pc)


def test_step_graph_checks_its_warmup(gpu):
    """A dirty solve workspace makes the graph's warm-up run abort: StepGraph
    raises there (it used to reset the flag and capture on the dirty words,
    so every replay gave a NaN PC), the words are re-zeroed, and the graph
    built afterwards replays the eager step bit for bit."""
    inp, gen = _bench_like_step(gpu, 3000, mosi=True)
    st = P.FusedStep(inp, gen.networks())
    s0, m0 = [t.clone() for t in st.run(check=True)]
    _set_word(st.solve_ws, ABORT, 1)
    with pytest.raises(RuntimeError, match="timed out"):
        P.StepGraph(st)
    assert not bool(st.solve_ws[:16].any())
    st.reset()
    g = P.StepGraph(st)
    for _ in range(3):
        s1, m1 = g.run(check=True)
        assert torch.equal(s0, s1) and torch.equal(m0, m1)
    assert not bool(st.solve_ws[:16].any())


def _train_call(dev, ws, flag, w, seed=3, n=256, d=300, h=100, epochs=2, B=32):
    g = torch.Generator(device=dev).manual_seed(seed)
    lat = torch.randn(n, d, generator=g, device=dev)
    lab = torch.randn(n, 1, generator=g, device=dev)
    perm = torch.cat([torch.randperm(n, generator=g, device=dev) for _ in range(epochs)])
    w1, b1, w2, b2 = [t.clone() for t in w]
    spe = (n + B - 1) // B
    step_loss = torch.full((spe * epochs,), -1.0, device=dev)
    L.call("mmb_mlp_train", L.ptr(lat), L.ptr(lab), L.ptr(perm), n, epochs, B, d, h, 1, 0.01,
           L.ptr(w1), L.ptr(b1), L.ptr(w2), L.ptr(b2), L.ptr(step_loss), None, None, None, 0, 1,
           0, None, L.ptr(ws), L.ptr(flag), L.stream_ptr())
    torch.cuda.synchronize()
    return (w1, b1, w2, b2), step_loss


@pytest.mark.parametrize("what,word,value", DIRTY, ids=[d[0] for d in DIRTY])
def test_mlp_train_dirty_workspace_aborts_and_recovers(gpu, what, word, value):
    """mmb_mlp_train (P = ceil(100 / 32) = 4 workgroups exchanging every
    mini-batch): a dirty workspace ends the launch with the flag set instead
    of training on half-exchanged outputs; a zeroed one trains bit-identically
    to a fresh run and is left zero."""
    d, h = 300, 100
    g = torch.Generator(device=gpu).manual_seed(1)
    w = (torch.randn(h, d, generator=g, device=gpu) * 0.05, torch.zeros(h, device=gpu),
         torch.randn(1, h, generator=g, device=gpu) * 0.1, torch.zeros(1, device=gpu))
    nws = L.query("mmb_mlp_workspace_bytes", d, h) // 4 + 4
    flag = torch.zeros(1, dtype=torch.int32, device=gpu)
    ws = torch.zeros(nws, dtype=torch.float32, device=gpu)
    p0, l0 = _train_call(gpu, ws, flag, w)
    assert int(flag.item()) == 0 and not bool(ws[:4].view(torch.int32).any())
    assert bool((l0 >= 0).all())
    ws.view(torch.int32)[word] = value
    _train_call(gpu, ws, flag, w)
    assert int(flag.item()) & L.MMB_FLAG_SYNC_TIMEOUT, what
    ws.zero_()
    flag.zero_()
    p1, l1 = _train_call(gpu, ws, flag, w)
    assert int(flag.item()) == 0
    assert torch.equal(l0, l1) and all(torch.equal(a, b) for a, b in zip(p0, p1))


def _perturb(inp, i):
    """Change every input of the step in place: frames rescaled (powers of two
    up and down, so the int8 Gram's column bounds must follow), ids rolled,
    word-table rows rescaled (the text cache must follow: in-place writes bump
    the version counter)."""
    f = (4.0, 0.25, 3.0)[i % 3]
    inp["audio"].mul_(f)
    inp["visual"].mul_(1.0 / f)
    inp["ids"].copy_(torch.roll(inp["ids"], shifts=1 + i, dims=0))
    inp["table"][: inp["table"].shape[0] // 2].mul_(f)


@pytest.mark.parametrize("mosi,n", [(True, 1 << 15), (False, 40_000), (False, 200_018)],
                         ids=["narrow_fused", "stream_project", "stream_project_dynamic_order"])
def test_graph_replay_int8_gram_on_changing_inputs(gpu, mosi, n):
    """>= 32,768 rows (GRAM_I8_MIN_ROWS): the captured step runs the stream
    kernel's column-bound partials, their reduction and the int8 Gram.  Each
    replay follows new inputs (rescaled frames and table rows, re-ordered ids)
    and equals an eager step on the same inputs bit for bit: SIF rows, MMB2
    rows, PC, column bounds -- a stale bound, hand-over word or text cache
    would show.  At 200,018 rows (>= 16 rounds of 48-row batches) the fused
    kernel runs in its dynamic batch order: the batch counter is re-zeroed by a
    kernel node on every replay."""
    if n > 100_000:
        assert (n + 47) // 48 >= 16 * min(256, L.cu_count(gpu))
    inp, gen = _bench_like_step(gpu, n, mosi=mosi, seed=93)
    st = P.FusedStep(inp, gen.networks())
    assert st.gram_i8 and (st.narrow_fused if mosi else st.stream_project)
    g = P.StepGraph(st)
    for i in range(3):
        _perturb(inp, i)
        s_g, m_g = [t.clone() for t in g.run(check=True)]
        pc_g, cm_g = st.pc.clone(), st.colmax.clone()
        ref = P.FusedStep(inp, gen.networks())
        s_e, m_e = ref.run(check=True)
        assert torch.equal(cm_g, ref.colmax), i
        assert torch.equal(pc_g, ref.pc), i
        assert torch.equal(s_g, s_e) and torch.equal(m_g, m_e), i
        del ref
    assert not bool(st.solve_ws[:16].any())


def test_text_cache_follows_a_new_weight_tensor(gpu):
    """The narrow fused kernel reads token weights from the text cache's copy:
    handing mm2_stream_project_narrow a DIFFERENT weight tensor with the same
    projection rebuilds the cache, so the rows equal the two-kernel step's
    with the new weights (the cache used to be keyed on the word table only)."""
    N, T, A, Vd, V = 3000, 20, 76, 48, 3016
    inp = synth.device_workload(N, T, V, A=A, Vd=Vd, seed=97, device=gpu)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(gpu)
    proj = P.MMB2Projection(gen.networks(), 300, A, Vd, T, gpu)
    args = (N, T, 300, A, Vd, inp["audio"], inp["visual"], proj, inp["ids"], inp["table"])
    x0, _, m0 = [t.clone() for t in P.mm2_stream_project_narrow(*args, inp["wtab"])]
    w2 = inp["wtab"].clone()
    w2[: V // 3] *= 2.5
    x1, aux1, m1 = P.mm2_stream_project_narrow(*args, w2)
    inp2 = dict(inp, wtab=w2)
    b = P.FusedStep(inp2, gen.networks(), narrow_fused=False)
    b.run(check=True)
    torch.cuda.synchronize()
    assert not torch.equal(m0, m1)
    from oracle import mmb2_oracle as M
    assert M.row_rel_err(x1.cpu().numpy(), b.x.cpu().numpy()) < 2e-6
    assert M.row_rel_err(m1.cpu().numpy(), b.mmb2.cpu().numpy()) < 2e-6
    assert torch.allclose(aux1[1], b.aux[1], rtol=1e-6, atol=0)


_RCCL_CHILD = r"""
import json, os, sys
sys.path[:0] = [os.environ["MMB_ROOT"], os.path.join(os.environ["MMB_ROOT"], "multimodal-baselines_amd")]
import torch, torch.distributed as dist
import distributed as D, models, pipeline as P, synth
rank, world, dev = D.init("nccl", force_group=True)
assert dist.is_initialized() and world == 1
inp = synth.device_workload(40_000, 40, 50_000, A=300, Vd=300, seed=99, device=dev)
torch.manual_seed(0)
gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(dev)
ar = D.allreduce_sum(force=True)
calls = []
def counted(t):
    calls.append(str(t.dtype))
    ar(t)
st = D.sharded_fused_step(inp, gen.networks(), n_total=40_000, row0=0, allreduce=counted)
s1, m1 = [t.clone() for t in st.run()]   # checked: check()'s flag all-reduce too
ref = P.FusedStep(inp, gen.networks())
s0, m0 = ref.run(check=True)
torch.cuda.synchronize()
out = {"backend": dist.get_backend(), "world": dist.get_world_size(), "calls": calls,
       "sif_equal": bool(torch.equal(s0, s1)), "mmb2_equal": bool(torch.equal(m0, m1)),
       "pc_equal": bool(torch.equal(ref.pc, st.pc)), "gram_equal": bool(torch.equal(ref.G, st.G))}
dist.destroy_process_group()
print(json.dumps(out), flush=True)
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_world_one_on_the_step_path(gpu):
    """The product FusedStep through distributed.init("nccl") with a forced
    RCCL all-reduce at world size 1 (a fresh child process: one process group
    per process): the Gram's f64 SUM and check()'s int32 flag-bit SUM go
    through RCCL, and rows, Gram and PC are bit-identical to the
    non-distributed step."""
    env = {**os.environ, "MMB_ROOT": ROOT, "WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0",
           "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_free_port())}
    r = subprocess.run([sys.executable, "-u", "-c", _RCCL_CHILD], env=env, capture_output=True,
                       text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["backend"] == "nccl" and out["world"] == 1
    assert out["calls"] == ["torch.float64", "torch.int32"], out["calls"]
    assert out["sif_equal"] and out["mmb2_equal"] and out["pc_equal"] and out["gram_equal"], out
