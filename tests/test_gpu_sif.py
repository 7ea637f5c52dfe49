"""GPU parity: SIF text path (a1-a5) through libmmb vs the reference fixtures and the oracle.

Bars (BASELINE.json north_star): a1 bit-exact; embeddings within
1e-5 row-relative (max_j |y - y_ref| / max_j |y_ref|) of the reference f64
output; the PC within 1e-8 of the reference's randomized-SVD PC.
"""
import numpy as np
import pytest
import torch

import pipeline as P
import sif
import sif_functions as SF
import synth
from oracle import mmb2_oracle as M
from oracle import sif_oracle as O

pytestmark = pytest.mark.gpu

SIF_CASES = ["g1_pom_valid", "g1_pom_test", "g2_mosi", "g3_gap"]
EMB_TOL = 1e-5


def regen_table(z):
    return synth.word_table(int(z["V"]), int(z["D"]), seed=int(z["table_seed"]),
                            common=float(z["common"]))


@pytest.mark.parametrize("case", SIF_CASES)
def test_seq2weight_bit_exact(gpu, golden, case):
    z = golden(case)
    w = sif.get_sentence_word_weights(z["ids"], z["weights"])
    assert w.dtype == np.float32 and np.array_equal(w, z["w"])


def test_seq2weight_mask_and_negative_ids(gpu, golden):
    z = golden("g1c_seq2weight")
    w = SF.seq2weight(z["seq"], z["mask"], z["weights"])
    assert np.array_equal(w, z["w"])


def test_seq2weight_out_of_range_raises(gpu):
    with pytest.raises(IndexError):
        SF.seq2weight(np.array([[0, 5]]), np.ones((1, 2)), np.ones(5))


@pytest.mark.parametrize("case", SIF_CASES)
def test_weighted_average(gpu, golden, case):
    z = golden(case)
    emb = SF.get_weighted_average(regen_table(z), z["ids"], z["w"])
    assert emb.dtype == np.float64 and emb.shape == z["emb"].shape
    assert M.row_rel_err(emb, z["emb"]) < 2e-6


def test_weighted_average_negative_ids_wrap(gpu, golden):
    z = golden("g1c_seq2weight")
    emb = SF.get_weighted_average(regen_table(z), z["seq"], z["w"])
    assert M.row_rel_err(emb, z["emb"]) < 2e-6


@pytest.mark.parametrize("case", SIF_CASES + ["g3b_npc2"])
def test_compute_pc_replays_randomized_svd(gpu, golden, case):
    """Device PC from the Gram == sklearn's randomized PC, also without a gap (g3)."""
    z = golden(case)
    npc = z["pc"].shape[0]
    pc = SF.compute_pc(z["emb"].astype(np.float64), npc)
    assert pc.shape == z["pc"].shape
    assert np.abs(pc - z["pc"]).max() < 1e-8


@pytest.mark.parametrize("case", SIF_CASES)
def test_sentence_embeddings_end_to_end(gpu, golden, case):
    z = golden(case)
    out = sif.get_sentence_embeddings(regen_table(z), z["weights"], z["ids"])
    assert out.dtype == np.float64
    assert M.row_rel_err(out, z["out"]) < EMB_TOL


def test_sif_embedding_with_given_weights(gpu, golden):
    z = golden("g2_mosi")
    p = SF.Params()
    p.rmpc = 1
    out = SF.SIF_embedding(regen_table(z), z["ids"], z["w"], p)
    assert M.row_rel_err(out, z["out"]) < EMB_TOL
    p.rmpc = 0
    emb = SF.SIF_embedding(regen_table(z), z["ids"], z["w"], p)
    assert M.row_rel_err(emb, z["emb"]) < 2e-6


def test_remove_pc_npc2(gpu, golden):
    z = golden("g3b_npc2")
    out = SF.remove_pc(z["emb"].astype(np.float64), 2)
    assert M.row_rel_err(out, z["out"]) < 1e-9


def test_empty_and_single_token_utterances(gpu):
    """Ragged edge cases: length-1 rows and rows of pure padding (count 0 -> nan, as numpy)."""
    V = 500
    E = synth.word_table(V, 300, seed=3)
    wt = synth.sif_weights(V, w0=0.0)
    ids = synth.token_ids(400, 12, V, seed=4, ragged=True)
    ids[0, 1:] = 0
    ids[1, :] = 0
    w = O.seq2weight(ids, np.ones(ids.shape), wt)
    ref = O.get_weighted_average(E, ids, w)  # row 1: 0/0 -> nan
    got = SF.get_weighted_average(E, ids, w)
    assert np.isnan(got[1]).all() and np.isnan(ref[1]).all()
    ok = ~np.isnan(ref).any(axis=1)
    assert M.row_rel_err(got[ok], ref[ok]) < 2e-6


@pytest.mark.parametrize("N,L,V", [(3000, 40, 20000), (700, 256, 5000)])
def test_sif_vs_oracle_mid_size(gpu, N, L, V):
    E = synth.word_table(V, 300, seed=N)
    wt = synth.sif_weights(V, w0=1.0)
    ids = synth.token_ids(N, L, V, seed=L, ragged=True)
    ref = O.get_sentence_embeddings(E, wt, ids)
    got = sif.get_sentence_embeddings(E, wt, ids)
    assert M.row_rel_err(got, ref) < EMB_TOL


@pytest.mark.parametrize("n_total,shards", [(5000, 4), (250, 2)])
def test_sharded_equals_unsharded_on_one_gpu(gpu, n_total, shards):
    """The multi-GPU decomposition on one device: per-shard Grams (and X^T Omega
    rows in the transposed branch, n_total < 300) summed as the all-reduce
    would, then the same solve — equals the unsharded PC and embeddings."""
    import distributed as D

    V = 8000
    E = torch.tensor(synth.word_table(V, 300, seed=11), device=gpu)
    wt = torch.tensor(synth.sif_weights(V), device=gpu, dtype=torch.float32)
    ids = torch.as_tensor(synth.token_ids(n_total, 30, V, seed=12, ragged=True), device=gpu)
    ref, pc_ref = P.sif_embeddings(E, ids, wtab32=wt, out_dtype=torch.float64)
    k = 1 + P.N_OVERSAMPLES
    parts, G, z0 = [], None, None
    for r in range(shards):
        row0, n = D.shard_range(n_total, shards, r)
        num, cnt = P.weighted_sum(E, P.narrow_ids(ids[row0:row0 + n]), wtab32=wt)
        g = P.gram(num, cnt)
        G = g if G is None else G + g
        if n_total < 300:
            om = P.omega(n_total, k, gpu)[row0:row0 + n].contiguous()
            zr = P.xt_omega(num, cnt, om)
            z0 = zr if z0 is None else z0 + zr
        parts.append((num, cnt))
    transposed = n_total < 300
    if not transposed:
        z0 = P.omega(300, k, gpu)
    pc = P.pc_solve(G, z0, 1, transposed)
    assert (pc - pc_ref).abs().max().item() < 1e-10
    out = torch.cat([P.remove_pc(num, cnt, pc, torch.float64) for num, cnt in parts])
    assert M.row_rel_err(out.cpu().numpy(), ref.cpu().numpy()) < 1e-9


def test_device_sif_properties_large(gpu):
    """Size-independent properties at a large N: the output is orthogonal to the
    removed PC, removal is idempotent, and two runs are bit-identical."""
    N, L, V = 200_000, 40, 100_000
    inp = synth.device_workload(N, L, V, A=4, Vd=4, seed=5, device=gpu)
    out1, pc = P.sif_embeddings(inp["table"], inp["ids"], wtab32=inp["wtab"], npc=1,
                                out_dtype=torch.float64)
    out2, _ = P.sif_embeddings(inp["table"], inp["ids"], wtab32=inp["wtab"], npc=1,
                               out_dtype=torch.float64)
    assert torch.equal(out1, out2)
    proj = (out1 @ pc.T).abs().max().item()
    assert proj < 1e-10 * out1.abs().max().item() * 300
    assert abs(torch.linalg.norm(pc).item() - 1.0) < 1e-12
    # idempotence: removing the same pc again changes nothing beyond rounding
    again = out1 - (out1 @ pc.T) * pc
    assert (again - out1).abs().max().item() < 1e-12


def test_two_phase_gram_equals_one_shot_and_fp64(gpu):
    """mmb_gram_part over row chunks + one mmb_gram_finish equals the one-shot
    mmb_gram and the exact f64 X^T X (products of f32 values are exact in
    f64; only the summation order differs)."""
    import mmb_lib as L

    n_plan, d = 4096, 300
    rng = np.random.default_rng(5)
    X = (rng.standard_normal((3 * n_plan - 100, d)) * 0.4 + 0.3).astype(np.float32)
    x = torch.tensor(X, device=gpu)
    ws = P.GramWorkspace(n_plan, d, gpu)
    G2 = torch.empty((d, d), dtype=torch.float64, device=gpu)
    for c, r0 in enumerate(range(0, x.shape[0], n_plan)):
        part = x[r0:r0 + n_plan]
        L.call("mmb_gram_part", L.ptr(part), None, part.shape[0], n_plan, d, int(c > 0),
               L.ptr(ws.buf), L.stream_ptr())
    L.call("mmb_gram_finish", n_plan, d, L.ptr(G2), 0, L.ptr(ws.buf), L.stream_ptr())
    G1 = P.gram(x, None)
    ref = X.astype(np.float64).T @ X.astype(np.float64)
    scale = np.abs(ref).max()
    assert np.abs(G2.cpu().numpy() - ref).max() / scale < 1e-13
    assert np.abs(G1.cpu().numpy() - ref).max() / scale < 1e-13
    with pytest.raises(L.MMBError):  # a chunk larger than the plan is rejected
        L.call("mmb_gram_part", L.ptr(x), None, x.shape[0], n_plan, d, 0, L.ptr(ws.buf),
               L.stream_ptr())


def test_compute_pc_float64_input_is_not_rounded(gpu, golden):
    """A float64 X that is not f32-representable takes the f64-row kernels
    (mmb_gram_f64 / mmb_xt_omega_f64 / mmb_pc_remove_f64): the PC and the
    removal match the reference's f64 randomized SVD to f64 rounding, where
    rounding X to f32 first would be ~1e-7 off.  Both sklearn branches."""
    for case in ("g2_mosi", "g1_pom_valid"):
        z = golden(case)
        rng = np.random.default_rng(3)
        X = z["emb"].astype(np.float64) * (1.0 + 1e-6 * rng.standard_normal(z["emb"].shape))
        assert not np.array_equal(X.astype(np.float32).astype(np.float64), X)
        ref_pc = O.compute_pc(X, 1)
        pc = SF.compute_pc(X, 1)
        assert np.abs(pc - ref_pc).max() < 1e-12
        out = SF.remove_pc(X, 1)
        assert M.row_rel_err(out, O.remove_pc(X, 1)) < 1e-12


@pytest.mark.parametrize("n", [1, 2, 5, 10, 11, 12])
def test_compute_pc_tiny_splits(gpu, n):
    """Splits smaller than the randomized-SVD block (n < npc + 10 = 11): the
    block is rank-deficient; the device solver must still give sklearn's PC."""
    rng = np.random.default_rng(n)
    g = rng.standard_normal(300)
    X = (0.4 * rng.standard_normal((n, 300)) + 0.3 * g).astype(np.float32).astype(np.float64)
    ref = O.compute_pc(X, 1)
    pc = SF.compute_pc(X, 1)
    assert np.isfinite(pc).all()
    assert np.abs(pc - ref).max() < 1e-8


def test_npc_limit_raises_value_error(gpu, golden):
    z = golden("g2_mosi")
    with pytest.raises(ValueError, match="npc"):
        SF.compute_pc(z["emb"].astype(np.float64), 7)
    assert SF.compute_pc(z["emb"].astype(np.float64), 6).shape == (6, 300)


def test_zero_weight_utterance_raises_like_reference(gpu):
    """An utterance whose SIF weights are all 0 makes the reference's
    TruncatedSVD raise ValueError (NaN row); so does the device path, while the
    plain weighted average keeps numpy's NaN row."""
    V = 500
    E = synth.word_table(V, 300, seed=3)
    wt = synth.sif_weights(V, w0=0.0)
    ids = synth.token_ids(400, 12, V, seed=4, ragged=True)
    ids[5, :] = 0
    with pytest.raises(ValueError, match="NaN"):
        sif.get_sentence_embeddings(E, wt, ids)
    w = O.seq2weight(ids, np.ones(ids.shape), wt)
    with pytest.raises(ValueError, match="NaN"):
        SF.compute_pc(SF.get_weighted_average(E, ids, w))


@pytest.mark.parametrize("n_total,shards", [(5000, 4), (250, 2), (1200, 3)])
def test_fused_step_sharded_with_fake_allreduce(gpu, n_total, shards):
    """The multi-GPU bench step, all ranks on one device: every shard runs the
    product FusedStep(n_total=..., row0=..., allreduce=fake) where `fake`
    adds the OTHER shards' Grams (and X^T Omega blocks in the transposed
    branch, n_total < 300) exactly where RCCL's all_reduce would.  The PC must
    equal the unsharded step's to 1e-10, the SIF rows to the removal's dot
    order, and the MMB2 rows bit for bit (they never cross shards)."""
    import distributed as D

    V = 8000
    inp = synth.device_workload(n_total, 40, V, seed=13, device=gpu)
    torch.manual_seed(0)
    import models

    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(gpu)
    whole = P.FusedStep(inp, gen.networks())
    s_ref, m_ref = [t.clone() for t in whole.run()]
    pc_ref = whole.pc.clone()

    def shard(r):
        row0, n = D.shard_range(n_total, shards, r)
        sl = {k: (v[row0:row0 + n] if k in ("ids", "audio", "visual") else v)
              for k, v in inp.items()}
        return row0, n, sl

    # pass 1: every shard's local contributions, in all_reduce call order
    local = []
    for r in range(shards):
        row0, n, sl = shard(r)
        got = []
        step = P.FusedStep(sl, gen.networks(), n_total=n_total, row0=row0,
                           allreduce=lambda t, got=got: got.append(t.clone()))
        step.run()
        step.check()  # sharded: its flag bits cross the ranks too
        local.append(got)
    n_calls = (2 if n_total < 300 else 1) + 1
    assert all(len(g) == n_calls for g in local)

    # pass 2: the fake all-reduce adds the other shards' tensors in rank order
    sif_parts, mm2_parts = [], []
    for r in range(shards):
        row0, n, sl = shard(r)
        calls = iter(range(n_calls))

        def fake(t, r=r, calls=calls):
            c = next(calls)
            tot = torch.zeros_like(t)
            for q in range(shards):
                tot += t if q == r else local[q][c]
            t.copy_(tot)

        step = P.FusedStep(sl, gen.networks(), n_total=n_total, row0=row0, allreduce=fake)
        trace = {}
        s, m = step.run(trace=trace)
        assert "allreduce" in trace
        assert (step.pc - pc_ref).abs().max().item() < 1e-10
        step.check()
        sif_parts.append(s.clone())
        mm2_parts.append(m.clone())
    assert torch.equal(torch.cat(mm2_parts), m_ref)
    assert M.row_rel_err(torch.cat(sif_parts).cpu().numpy(), s_ref.cpu().numpy()) < 1e-6


@pytest.mark.parametrize("value", [float("inf"), float("nan")])
@pytest.mark.parametrize("gram_kind", ["i8", "f64"])
def test_nonfinite_table_row_raises(gpu, value, gram_kind):
    """A non-finite word-table entry used with a nonzero weight makes that
    utterance's a2 row non-finite; the reference's TruncatedSVD rejects the
    split (ValueError, sif_functions.py:65).  The int8 Gram carries it: the
    column bound keeps NaN / inf (max on the bits), and a non-finite bound
    writes NaN into G, so the PC is NaN and check() raises -- as with the
    exact f64 Gram."""
    import models

    inp = synth.device_workload(2000, 40, 8000, seed=19, device=gpu)
    inp["table"][11, 17] = value
    inp["ids"][123, 5] = 11
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(gpu)
    step = P.FusedStep(inp, gen.networks(), gram_kind=gram_kind)
    step.run()
    if gram_kind == "i8":
        cm = step.colmax.cpu().numpy().view(np.float32)
        assert not np.isfinite(cm[17]) and np.isfinite(np.delete(cm, 17)).all()
    with pytest.raises(ValueError, match="NaN or infinity"):
        step.check()


@pytest.mark.parametrize("bad,err", [("id_range", IndexError), ("zero_weight", ValueError),
                                     ("none", None)])
def test_sharded_checked_step_raises_on_every_rank(gpu, bad, err):
    """distributed.sharded_fused_step returns a checked step: a token id >= V
    (numpy's IndexError, sif_functions.py:55) or an all-zero-weight utterance
    (TruncatedSVD's ValueError on the NaN row, sif_functions.py:65) on ONE
    shard raises on EVERY shard -- the flag bits are summed by the step's
    all-reduce, and the zero-weight row's NaN reaches every shard's PC through
    the int8 Gram (a non-finite column bound makes G NaN) -- so no rank is left
    waiting in the next all-reduce.  Three shards on one device, RCCL's
    all-reduce replaced by a fake that adds the other shards' tensors in call
    order (recorded in a first pass)."""
    import distributed as D
    import models

    n_total, shards, V = 3000, 3, 8000
    inp = synth.device_workload(n_total, 40, V, seed=17, device=gpu)
    if bad == "id_range":
        inp["ids"][1500, 3] = V + 5  # shard 1's rows are [1000, 2000)
    elif bad == "zero_weight":
        inp["wtab"][7] = 0.0
        inp["ids"][1500] = 7
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(gpu)

    def shard(r):
        row0, n = D.shard_range(n_total, shards, r)
        return row0, {k: (v[row0:row0 + n] if k in ("ids", "audio", "visual") else v)
                      for k, v in inp.items()}

    local = []
    for r in range(shards):  # pass 1: each shard's own all-reduce operands, in call order
        row0, sl = shard(r)
        got = []
        step = D.sharded_fused_step(sl, gen.networks(), n_total, row0,
                                    allreduce=lambda t, got=got: got.append(t.clone()))
        try:
            step.run()
        except (IndexError, ValueError):
            assert r == 1 and err is not None  # only the shard holding the bad row
        local.append(got)
    assert all(len(g) == 2 for g in local)  # the Gram, then check()'s flag bits
    for r in range(shards):  # pass 2: the fake all-reduce sums over the shards
        row0, sl = shard(r)
        calls = iter(range(2))

        def fake(t, r=r, calls=calls):
            c = next(calls)
            tot = torch.zeros_like(t)
            for q in range(shards):
                tot += t if q == r else local[q][c]
            t.copy_(tot)

        step = D.sharded_fused_step(sl, gen.networks(), n_total, row0, allreduce=fake)
        if err is None:
            step.run()
            assert bool(torch.isfinite(step.pc).all())
        else:
            with pytest.raises(err):
                step.run()


@pytest.mark.parametrize("n,seed,scale", [(320, 0, 1.0), (5000, 1, 1.0), (70_000, 2, 1e-3),
                                          (1000, 3, 1e4), (7, 4, 1.0)])
def test_gram_i8_vs_sliced_oracle_and_f64(gpu, n, seed, scale):
    """mmb_gram_i8 (int8 digits, exact integer level sums) against its CPU
    restatement oracle.sif_oracle.sliced_gram (same digits; f64 summation
    order only) and the exact f64 Gram (2e-9; heavy-tailed t(3) columns), rows
    past 64-row chunks, tiny and huge magnitudes, a column of zeros."""
    from oracle import sif_oracle as O

    rng = np.random.default_rng(seed)
    x = (rng.standard_t(3, size=(n, 300)) * scale).astype(np.float32)
    x[:, 17] = 0.0
    xt = torch.tensor(x, device=gpu)
    cm = P.colmax(xt)
    assert np.array_equal(cm.cpu().numpy().view(np.float32), np.abs(x).max(0))
    G = P.gram_i8(xt, cm).cpu().numpy()
    ref = O.sliced_gram(x)
    exact = x.astype(np.float64).T @ x.astype(np.float64)
    assert np.abs(G - ref).max() <= 1e-13 * np.abs(ref).max()
    assert np.abs(G - exact).max() <= 2e-9 * np.abs(exact).max()
    assert np.array_equal(G, G.T)


def test_gram_i8_blocks_past_int32_range_limit(gpu):
    """mmb_gram_i8 sums each range's digit-pair levels in int32 (exact for
    ranges of <= 32768 rows) and cuts calls above 128 such ranges
    (4,194,304 rows) into blocks whose reductions accumulate into G: a call
    just past one block (narrow rows, d = 16), and one with accumulate=True
    on top of a previous G, against the sliced restatement and the exact
    f64 Gram."""
    from oracle import sif_oracle as O

    n = 128 * 32768 + 1000
    g = torch.Generator(device=gpu).manual_seed(11)
    xt = (torch.randn(n, 16, generator=g, device=gpu) * 0.7 + 0.2).contiguous()
    xt[: n // 3] *= 3.0
    cm = P.colmax(xt)
    G = P.gram_i8(xt, cm)
    G2 = P.gram_i8(xt[:5000], cm, G.clone(), accumulate=True)
    x = xt.cpu().numpy()
    ref = O.sliced_gram(x, cm.cpu().numpy().view(np.float32))
    exact = x.astype(np.float64).T @ x.astype(np.float64)
    Gn = G.cpu().numpy()
    assert np.abs(Gn - ref).max() <= 1e-13 * np.abs(ref).max()
    assert np.abs(Gn - exact).max() <= 2e-9 * np.abs(exact).max()
    ref2 = ref + O.sliced_gram(x[:5000], cm.cpu().numpy().view(np.float32))
    assert np.abs(G2.cpu().numpy() - ref2).max() <= 1e-13 * np.abs(ref2).max()


def test_gram_i8_pc_on_golden_splits(gpu, golden):
    """The PC solved from the int8 Gram stays within 1e-9 of the reference's
    TruncatedSVD component on the golden splits (gap-free g3 and npc = 2
    included)."""
    for case in ("g2_mosi", "g3_gap", "g3b_npc2"):
        z = golden(case)
        x = torch.tensor(z["emb"], device=gpu)
        npc = z["pc"].shape[0]
        G = P.gram_i8(x, P.colmax(x))
        pc = P.pc_solve(G, P.omega(300, npc + 10, gpu), npc, False).cpu().numpy()
        assert np.abs(pc - z["pc"]).max() < 1e-9, case
