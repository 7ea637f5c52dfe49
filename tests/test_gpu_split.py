"""GPU parity of the few-long-rows stream path (mmb_mm2_stream_split, r06).

configs[2] at its real sizes (POM's splits: 100 / 203 transcripts of 1089 /
1357 tokens, simplesif.py:308-311) puts one workgroup per utterance on the
chip with the plain stream kernel; the split path cuts each utterance into P
token / frame ranges (their own workgroups) and adds the P partials in fixed
part order.  Checked here:
  * parts = 1 is the one-workgroup kernel bit for bit (same slot order);
  * any P: x, the s row, aux within the f32 order of the token / frame sums
    (1e-6 row-relative; counts exact), deterministic across launches, ids
    gathered or dense text, fp32 or fp16 hi / lo s, scalar-width frames;
  * the FusedStep with the split stream (and the projection forked beside
    the PC solve) equals the one-workgroup step to the removal's dot order,
    and both meet the oracle (sif_functions / sif2, 1e-5);
  * the split-K projection (mmb_mm2_project_x3_split) against the one-pass
    kernel: MMB2 rows to the K sum's f32 order, the fused PC removal's rows
    bit for bit (they depend on x and the PC only), ragged row tiles.
"""
import numpy as np
import pytest
import torch

import mmb_lib as L
import models
import pipeline as P
import synth
from oracle import mmb2_oracle as M
from oracle import sif_oracle as O

pytestmark = pytest.mark.gpu


def _pom(golden, case, n, A, Vd, seed, dev):
    """The reference's own POM split ids (pom_valid_ids 100 x 1089 /
    pom_test_ids 203 x 1357, g11) and weights, the seeded V = 7763 table,
    word-aligned frames set to -10 past each transcript's last token."""
    z = golden("g11_pom_splits")
    ids = z[f"{case}_ids"][:n]
    N, T = ids.shape
    E = synth.word_table(len(z["weights"]), 300, seed=int(z["table_seed"]))
    last = np.where(ids != 0, np.arange(T)[None, :], -1).max(1)
    pad = np.arange(T)[None, :] > last[:, None]
    audio = synth.frames(N, T, A, seed=seed)
    visual = synth.frames(N, T, Vd, seed=seed + 1)
    audio[pad] = -10.0
    visual[pad] = -10.0
    inp = {"table": torch.tensor(E, device=dev),
           "wtab": torch.tensor(z["weights"], device=dev, dtype=torch.float32),
           "ids": torch.as_tensor(ids, dtype=torch.int32, device=dev),
           "audio": torch.tensor(audio, device=dev), "visual": torch.tensor(visual, device=dev)}
    return inp, (E, z["weights"], ids, audio, visual)


def _stream(inp, s_half, split=None, parts=0, dense=False, colmax=False):
    n, t = inp["ids"].shape
    d, a, vd = 300, inp["audio"].shape[-1], inp["visual"].shape[-1]
    dev = inp["audio"].device
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    cm = torch.zeros(d, dtype=torch.int32, device=dev) if colmax else None
    cws = (torch.empty(L.query("mmb_mm2_colmax_ws_bytes", d), dtype=torch.uint8, device=dev)
           if colmax else None)
    kw = dict(ids32=inp["ids"], table=inp["table"], wtab32=inp["wtab"])
    if dense:
        ids = inp["ids"].long()
        text = inp["table"][ids].contiguous()
        kw = dict(text_dense=text, emb_dense=text, w_dense=inp["wtab"][ids].contiguous())
    x, s, aux = P.mm2_stream(n, t, d, a, vd, inp["audio"], inp["visual"], flag=flag,
                             s_half=s_half, colmax=cm, colmax_ws=cws, split=split, parts=parts, **kw)
    torch.cuda.synchronize()
    return [v.clone() for v in (x, s, aux, flag)] + ([cm.clone()] if colmax else [])


def _s_f32(s, aux, s_half):
    """The fp32 sums behind an s buffer (fp16 hi + lo over the row scale)."""
    if not s_half:
        return s.double()
    kp = s.shape[1] // 2
    return (s[:, :kp].double() + s[:, kp:].double()) / aux[2].double()[:, None]


@pytest.mark.parametrize("case,n,A,Vd", [("valid", 100, 300, 300),
                                         ("test", 203, 300, 300),
                                         ("test", 40, 46, 37)])
def test_split_stream_vs_one_workgroup(gpu, golden, case, n, A, Vd):
    inp, _ = _pom(golden, case, n, A, Vd, seed=90, dev=gpu)
    N, T = inp["ids"].shape
    assert N <= L.cu_count(gpu) and P.split_parts(N, T) >= 1
    for s_half in (True, False):
        ref = _stream(inp, s_half, colmax=True)  # one workgroup per utterance
        ws = P.split_ws(N, T, 300, A, Vd, gpu, parts=33)
        # one part: the same kernel order, bit for bit
        one = _stream(inp, s_half, split=ws, parts=1, colmax=True)
        for r, g in zip(ref, one):
            assert torch.equal(r, g)
        for parts in (0, 2, 7, 33):  # (0: the automatic plan)
            got = _stream(inp, s_half, split=ws, parts=parts, colmax=True)
            again = _stream(inp, s_half, split=ws, parts=parts, colmax=True)
            for g, h in zip(got, again):  # fixed part order: deterministic
                assert torch.equal(g, h), parts
            x0, s0, a0, f0, c0 = ref
            x1, s1, a1, f1, c1 = got
            assert M.row_rel_err(x1.cpu().numpy(), x0.cpu().numpy()) < 1e-6, parts
            assert torch.equal(a1[0], a0[0]) and int(f1.item()) == int(f0.item()) == 0
            assert (a1[1] - a0[1]).abs().max().item() <= 1e-6 * a0[1].abs().max().item()
            assert (a1[2] == a0[2]).float().mean().item() > 0.95  # powers of two
            q0, q1 = _s_f32(s0, a0, s_half), _s_f32(s1, a1, s_half)
            assert M.row_rel_err(q1.cpu().numpy(), q0.cpu().numpy()) < 1e-6, parts
            # the column bounds are the max |x| bits of the rows written
            cm = x1.abs().amax(0).contiguous().view(torch.int32)
            assert torch.equal(c1, cm)


def test_split_stream_dense_text(gpu, golden):
    """The dense-text form (the gpu2 drop-in's call shape) through the split
    path against the gathered form and the one-workgroup kernel."""
    inp, _ = _pom(golden, "valid", 64, 300, 300, seed=91, dev=gpu)
    N, T = inp["ids"].shape
    ws = P.split_ws(N, T, 300, 300, 300, gpu)
    ref = _stream(inp, True, dense=True)
    got = _stream(inp, True, split=ws, dense=True)
    assert M.row_rel_err(got[0].cpu().numpy(), ref[0].cpu().numpy()) < 1e-6
    q0, q1 = _s_f32(ref[1], ref[2], True), _s_f32(got[1], got[2], True)
    assert M.row_rel_err(q1.cpu().numpy(), q0.cpu().numpy()) < 1e-6
    gath = _stream(inp, True, split=ws)
    assert M.row_rel_err(gath[0].cpu().numpy(), got[0].cpu().numpy()) < 1e-6


def test_split_stream_flags_and_bounds(gpu, golden):
    """Out-of-range ids are flagged and contribute zero rows, an utterance
    whose weights are all zero is flagged (NaN row, as numpy) -- as the
    one-workgroup kernel; an undersized scratch is refused."""
    inp, _ = _pom(golden, "valid", 50, 300, 300, seed=92, dev=gpu)
    N, T = inp["ids"].shape
    inp["ids"][3, 700] = inp["table"].shape[0] + 5
    inp["ids"][9, :] = 0
    inp["wtab"] = inp["wtab"].clone()
    inp["wtab"][0] = 0.0  # utterance 9: every token id 0 with weight 0
    ws = P.split_ws(N, T, 300, 300, 300, gpu)
    ref = _stream(inp, True)
    got = _stream(inp, True, split=ws)
    assert int(got[3].item()) == int(ref[3].item()) == (L.MMB_FLAG_ID_RANGE | L.MMB_FLAG_ZERO_WEIGHTS)
    assert bool(torch.isnan(got[0][9]).all()) and bool(torch.isnan(ref[0][9]).all())
    ok = torch.ones(N, dtype=torch.bool, device=gpu)
    ok[9] = False
    assert M.row_rel_err(got[0][ok].cpu().numpy(), ref[0][ok].cpu().numpy()) < 1e-6
    with pytest.raises(L.MMBError):
        _stream(inp, True, split=ws[:1024])


@pytest.mark.parametrize("mode", ["eager", "graph"])
def test_split_step_vs_one_workgroup_step_and_oracle(gpu, golden, mode):
    """configs[2]'s step at the real valid-split size: the split stream and
    the forked projection (the default for these shapes) against the
    one-workgroup stream with the removal fused into the projection: MMB2
    rows and the a2 rows x to the stream's f32 sum order (1e-6), the PC to
    1e-7, the PC-removed rows to 1e-5; both within 1e-5 of the oracle."""
    inp, (E, wt, ids, audio, visual) = _pom(golden, "valid", 100, 300, 300, seed=93, dev=gpu)
    torch.manual_seed(4)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(gpu)
    new = P.FusedStep(inp, gen.networks())
    assert new.split is not None and new.fork is not None
    old = P.FusedStep(inp, gen.networks(), split_stream=False, fork_projection=False)
    assert old.split is None and old.fork is None and old.fused_remove
    s0, m0 = [t.clone() for t in old.run(check=True)]
    if mode == "graph":
        g = P.StepGraph(new)
        for _ in range(2):
            s1, m1 = g.run(check=True)
    else:
        s1, m1 = new.run(check=True)
    torch.cuda.synchronize()
    assert M.row_rel_err(m1.cpu().numpy(), m0.cpu().numpy()) < 1e-6
    assert M.row_rel_err(new.x.cpu().numpy(), old.x.cpu().numpy()) < 1e-6
    # n < d: sklearn's transposed branch, whose PC moves with the rows' f32
    # sum order by ~1e-8; the removed rows are small beside x, so their
    # relative difference is that of the PC (the bar is the north star's)
    assert (new.pc - old.pc).abs().max().item() < 1e-7
    assert M.row_rel_err(s1.cpu().numpy(), s0.cpu().numpy()) < 1e-5
    ref_sif = O.get_sentence_embeddings(E, wt, ids)
    assert M.row_rel_err(s1.cpu().numpy(), ref_sif) < 1e-5
    r = np.arange(0, 100, 3)
    sw = np.where(ids[r] >= 0, wt.astype(np.float32)[ids[r]], 0).astype(np.float32)
    text = E[ids[r]]
    ref_mm2 = M.estimate_embedding_overall_gpu2(M.concat_inputs(text, audio[r], visual[r]),
                                                 M.params_from_module(gen.cpu()), sw, text)
    assert M.row_rel_err(m1[torch.as_tensor(r, device=gpu)].cpu().numpy(), ref_mm2) < 1e-5


@pytest.mark.parametrize("n", [2, 5, 100, 129, 203, 700, 1000])
def test_split_k_projection_vs_one_pass(gpu, n):
    inp = synth.device_workload(n, 40, 5000, A=300, Vd=300, seed=60 + n, device=gpu)
    torch.manual_seed(3)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(gpu)
    st = P.FusedStep(inp, gen.networks(), stream_project=False, fork_projection=False,
                     split_stream=False)
    st.run(check=True)
    proj, s_, x, aux = st.proj, st.s, st.x, st.aux_of(0)
    pc = st.pc.clone()
    ref = P.mm2_project(s_, x, aux, proj).clone()
    sif_ref = torch.empty_like(x)
    ref2 = P.mm2_project(s_, x, aux, proj, pc=pc, sif_out=sif_ref).clone()
    assert torch.equal(ref, ref2)
    for slices in (0, 2, 3, 7, 57):
        ws = torch.empty(max(16, L.query("mmb_mm2_project_x3_split_ws_bytes", n, proj.kp, slices)),
                         dtype=torch.uint8, device=gpu)
        got = P.mm2_project(s_, x, aux, proj, split=ws, slices=slices).clone()
        again = P.mm2_project(s_, x, aux, proj, split=ws, slices=slices).clone()
        sif = torch.empty_like(x)
        got2 = P.mm2_project(s_, x, aux, proj, pc=pc, sif_out=sif, split=ws, slices=slices)
        torch.cuda.synchronize()
        assert torch.equal(got, again) and torch.equal(got, got2), slices
        assert torch.equal(sif, sif_ref), slices
        assert M.row_rel_err(got.cpu().numpy(), ref.cpu().numpy()) < 1e-6, slices
