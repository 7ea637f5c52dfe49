"""GPU parity: closed-form MMB2 (a7/a8) through libmmb vs the reference fixtures and the oracle.

Bar: 1e-5 row-relative against the reference's float64 evaluation of
sif2.estimate_embedding_overall_gpu2 (the reference's own fp32 run meets the
same bar, test_oracle_golden.py::test_mmb2_oracle).
"""
import numpy as np
import pytest
import torch

import mmb_lib as L
import models
import pipeline as P
import sif2
import synth
from oracle import mmb2_oracle as M
from oracle import sif_oracle as O

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _inputs(z, dev):
    A, Vd, V = int(z["A"]), int(z["Vd"]), int(z["V"])
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None, frozen_weights=True)
    E = synth.word_table(V, 300, seed=int(z["table_seed"]))
    ids = z["ids"]
    N, T = ids.shape
    pe = float(z["pad_frac"])
    audio = synth.frames(N, T, A, seed=int(z["audio_seed"]), pad_frac=pe)
    visual = synth.frames(N, T, Vd, seed=int(z["visual_seed"]), pad_frac=pe)
    return gen, E, ids, audio, visual, z["weights"]


def _drop_in_call(gen, E, ids, audio, visual, weights, dev):
    """The --time_test call site (simplesif.py:820-875) with our sif2."""
    word_embeddings = torch.tensor(E, device=dev)
    wt = torch.tensor(weights, device=dev, dtype=torch.float32)
    text_id = torch.as_tensor(ids, dtype=torch.long, device=dev)
    text = word_embeddings[text_id]
    au = torch.tensor(audio, device=dev)
    vi = torch.tensor(visual, device=dev)
    data = {"text": text, "audio": au, "visual": vi,
            "audiovisual": torch.cat([au, vi], -1), "textaudio": torch.cat([text, au], -1),
            "textvisual": torch.cat([text, vi], -1),
            "textaudiovisual": torch.cat([text, au, vi], -1)}
    masks = {k: None for k in list(data) + list(sif2.KEYS)}
    g = gen.to(dev)
    nets = {k: (g.embed2out[k]["mu"], g.embed2out[k]["log_sigma"]) for k in sif2.KEYS}
    sw = torch.gather(wt.expand(len(ids), -1), 1, text_id) * (text_id >= 0)
    with torch.no_grad():
        return sif2.estimate_embedding_overall_gpu2(data, masks, nets, sw, text)


@pytest.mark.parametrize("case", ["g4_mmb2_mosi", "g4_mmb2_syn"])
def test_gpu2_drop_in_vs_reference(gpu, golden, case):
    z = golden(case)
    gen, E, ids, audio, visual, weights = _inputs(z, gpu)
    cs = _drop_in_call(gen, E, ids, audio, visual, weights, gpu)
    assert cs.shape == (len(ids), 300) and cs.dtype == torch.float32
    assert M.row_rel_err(cs.cpu().numpy(), z["cs_f64"]) < TOL


@pytest.mark.parametrize("case", ["g4_mmb2_mosi", "g4_mmb2_syn"])
def test_fused_id_path_equals_dense_path(gpu, golden, case):
    z = golden(case)
    gen, E, ids, audio, visual, weights = _inputs(z, gpu)
    dense = _drop_in_call(gen, E, ids, audio, visual, weights, gpu)
    n, t = ids.shape
    A, Vd = audio.shape[-1], visual.shape[-1]
    table = torch.tensor(E, device=gpu)
    wtab = torch.tensor(weights, device=gpu, dtype=torch.float32)
    ids32 = torch.as_tensor(ids, dtype=torch.int32, device=gpu)
    au, vi = torch.tensor(audio, device=gpu), torch.tensor(visual, device=gpu)
    proj = P.MMB2Projection(gen.to(gpu).networks(), 300, A, Vd, t, gpu)
    # the drop-in's launch choices (sif2.py): split stream for a few long
    # rows, split-K projection for a few rows -- the same sum orders
    split = (P.split_ws(n, t, 300, A, Vd, gpu)
             if t > 64 and 0 < n <= L.cu_count(gpu) else None)
    num, s, aux = P.mm2_stream(n, t, 300, A, Vd, au, vi, ids32=ids32, table=table, wtab32=wtab,
                               split=split)
    fused = P.mm2_project(s, num, aux, proj, split=P.project_split_ws(n, proj.kp, gpu))
    if max(A, Vd) <= 128:  # the narrow-frame kernel: frame sums in another f32 order
        assert M.row_rel_err(fused.cpu().numpy(), dense.cpu().numpy()) < 1e-6
    else:
        assert torch.equal(fused, dense)


FP32_RATIO = 5.0  # measured 2.3-4.2x (r03d, tools/precision_probe.py)


def _row_errs(y, ref):
    return np.abs(y - ref).max(1) / np.abs(ref).max(1)


@pytest.mark.parametrize("case", ["g4_mmb2_mosi", "g4_mmb2_syn"])
def test_compensated_arithmetic_vs_reference_fp32(gpu, golden, case):
    """The MMB2 rows of the compensated paths (fp16 hi/lo x3 products with
    fp32 accumulation: the gpu2 drop-in's projection and the fused bench
    kernel) against the reference's own fp32 run of the same inputs
    (cs_f32, recorded from sif2.py:164-208 on the CPU), both measured from
    the reference's f64 rows: the worst row of ours stays within
    FP32_RATIO x the reference's worst fp32 row, and no worse than our
    exact-product fp32-MFMA projection (so the fp16 split is not what limits
    it: the closed form's per-utterance frame sums in f32 are)."""
    z = golden(case)
    gen, E, ids, audio, visual, weights = _inputs(z, gpu)
    ref64 = z["cs_f64"]
    e_ref = _row_errs(z["cs_f32"].astype(np.float64), ref64).max()
    drop = _drop_in_call(gen, E, ids, audio, visual, weights, gpu).cpu().numpy()
    n, t = ids.shape
    inputs = {"table": torch.tensor(E, device=gpu),
              "wtab": torch.tensor(weights, device=gpu, dtype=torch.float32),
              "ids": torch.as_tensor(ids, dtype=torch.int32, device=gpu),
              "audio": torch.tensor(audio, device=gpu), "visual": torch.tensor(visual, device=gpu)}
    step = P.FusedStep(inputs, gen.to(gpu).networks(), stream_project=True)
    assert step.stream_project
    fused = step.run()[1].cpu().numpy()
    A, Vd = audio.shape[-1], visual.shape[-1]
    num, s32, aux = P.mm2_stream(n, t, 300, A, Vd, inputs["audio"], inputs["visual"],
                                 ids32=inputs["ids"], table=inputs["table"],
                                 wtab32=inputs["wtab"], s_half=False)
    p32 = P.mm2_project(s32, num, aux, step.proj).cpu().numpy()
    e_drop = _row_errs(drop.astype(np.float64), ref64).max()
    e_fused = _row_errs(fused.astype(np.float64), ref64).max()
    e_p32 = _row_errs(p32.astype(np.float64), ref64).max()
    assert e_drop <= FP32_RATIO * e_ref and e_fused <= FP32_RATIO * e_ref, (e_drop, e_fused, e_ref)
    assert max(e_drop, e_fused) <= 1.1 * e_p32, (e_drop, e_fused, e_p32)
    if P.narrow_fused_supported(t, 300, A, Vd, E.shape[0]):
        # the narrow fused step (per-word text projection, f64-rounded P rows)
        nf = P.FusedStep(inputs, gen.to(gpu).networks())
        assert nf.narrow_fused
        e_nf = _row_errs(nf.run(check=True)[1].cpu().numpy().astype(np.float64), ref64).max()
        assert e_nf <= FP32_RATIO * e_ref, (e_nf, e_ref)


def test_compensated_arithmetic_vs_fp32_on_config3_sample(gpu):
    """The same pin on a sample of the configs[3] workload (40 frames, 3 x
    300-d, Zipf ids, V = 400k): the fused kernel's rows against the oracle's
    f64 closed form, next to the oracle's fp32 evaluation of the reference's
    formula (numpy float32, sif2.py:164-208 step by step) -- ours within
    FP32_RATIO x of that fp32 error."""
    n = 512
    inp = synth.device_shard(0, n, 40, 400_000, seed=1000, device=gpu)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(gpu)
    step = P.FusedStep(inp, gen.networks())
    fused = step.run(check=True)[1].cpu().numpy().astype(np.float64)
    ids = inp["ids"].long().cpu().numpy()
    E = inp["table"].cpu().numpy()
    wt = inp["wtab"].cpu().numpy()
    sw = wt[ids].astype(np.float32)
    text = E[ids]
    au, vi = inp["audio"].cpu().numpy(), inp["visual"].cpu().numpy()
    params = M.params_from_module(gen.cpu())
    cat = M.concat_inputs(text, au, vi)
    ref64 = M.estimate_embedding_overall_gpu2(cat, params, sw, text)
    ref32 = M.estimate_embedding_overall_gpu2(cat, params, sw, text, dtype=np.float32)
    e_ref = _row_errs(ref32.astype(np.float64), ref64).max()
    e_fused = _row_errs(fused, ref64).max()
    assert e_fused <= FP32_RATIO * e_ref, (e_fused, e_ref)
    assert e_fused < TOL


def test_calc_weights(gpu, golden):
    z = golden("g4_mmb2_mosi")
    gen, E, ids, audio, visual, weights = _inputs(z, gpu)
    m = gen.embed2out["audio"]
    qm, qs = sif2.calc_weights(torch.tensor(audio[:4], device=gpu), m["mu"].bias.to(gpu),
                               m["log_sigma"].bias.to(gpu), None)
    np.testing.assert_allclose(qm.cpu().numpy(), z["calc_qm_audio"], rtol=2e-6, atol=1e-6)
    np.testing.assert_allclose(qs.cpu().numpy(), z["calc_qs_audio"], rtol=2e-6, atol=1e-5)


def test_missing_combination_raises(gpu, golden):
    z = golden("g4_mmb2_mosi")
    gen, E, ids, audio, visual, weights = _inputs(z, gpu)
    with pytest.raises(KeyError):
        sif2.estimate_embedding_overall_gpu2({}, {}, {"audio": None}, None, None)


def test_single_utterance_errors_like_reference(gpu, golden):
    z = golden("g4_mmb2_mosi")
    gen, E, ids, audio, visual, weights = _inputs(z, gpu)
    with pytest.raises(IndexError):
        _drop_in_call(gen, E, ids[:1], audio[:1], visual[:1], weights, gpu)


@pytest.mark.parametrize("N,T,A,Vd", [(2048, 40, 300, 300), (1000, 20, 78, 50), (256, 300, 300, 300),
                                     (100, 130, 78, 50)])
def test_fused_step_vs_oracle(gpu, N, T, A, Vd):
    """Both outputs of the bench step against the oracle at a mid size
    (incl. feature widths that are not multiples of 4: scalar-load variants, and
    T > 64: the POM-shape workgroup-per-utterance stream kernel)."""
    from oracle import sif_oracle as O

    V = 30_000
    torch.manual_seed(1)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None)
    E = synth.word_table(V, 300, seed=2)
    wt = synth.sif_weights(V, w0=1.0)
    ids = synth.token_ids(N, T, V, seed=3, ragged=True)
    audio = synth.frames(N, T, A, seed=4, pad_frac=0.2)
    visual = synth.frames(N, T, Vd, seed=5, pad_frac=0.2)
    inputs = {"table": torch.tensor(E, device=gpu),
              "wtab": torch.tensor(wt, device=gpu, dtype=torch.float32),
              "ids": torch.as_tensor(ids, dtype=torch.int32, device=gpu),
              "audio": torch.tensor(audio, device=gpu), "visual": torch.tensor(visual, device=gpu)}
    step = P.FusedStep(inputs, gen.to(gpu).networks())
    sif_out, mm2_out = step.run()
    ref_sif = O.get_sentence_embeddings(E, wt, ids)
    assert M.row_rel_err(sif_out.cpu().numpy(), ref_sif) < TOL
    sw = np.where(ids >= 0, wt.astype(np.float32)[ids], 0).astype(np.float32)
    text = E[ids]
    ref_mm2 = M.estimate_embedding_overall_gpu2(M.concat_inputs(text, audio, visual),
                                                 M.params_from_module(gen.cpu()), sw, text)
    assert M.row_rel_err(mm2_out.cpu().numpy(), ref_mm2) < TOL


@pytest.mark.parametrize("scale,pad", [(1.0, 0.0), (100.0, 0.3), (1e-3, 0.0)])
def test_fp16_split_projection_vs_fp32_and_oracle(gpu, scale, pad):
    """The fp16 hi/lo split GEMM (bench path) and the fp32-MFMA GEMM both meet
    the 1e-5 bar, also for frames of very large / very small magnitude (the
    per-row and per-column power-of-2 scaling keeps fp16 in range).  N=700 is
    not a multiple of the 128-row tile (clamped tail rows)."""
    N, T, A, Vd, V = 700, 40, 300, 300, 5000
    torch.manual_seed(3)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None)
    E = synth.word_table(V, 300, seed=4) * np.float32(scale)
    wt = synth.sif_weights(V)
    ids = synth.token_ids(N, T, V, seed=5, ragged=True)
    audio = synth.frames(N, T, A, seed=6, pad_frac=pad) * np.float32(scale)
    visual = synth.frames(N, T, Vd, seed=7, pad_frac=pad) * np.float32(scale)
    ids32 = torch.as_tensor(ids, dtype=torch.int32, device=gpu)
    au, vi = torch.tensor(audio, device=gpu), torch.tensor(visual, device=gpu)
    proj = P.MMB2Projection(gen.to(gpu).networks(), 300, A, Vd, T, gpu)
    table = torch.tensor(E, device=gpu)
    wtab = torch.tensor(wt, device=gpu, dtype=torch.float32)
    num, s, aux = P.mm2_stream(N, T, 300, A, Vd, au, vi, ids32=ids32, table=table, wtab32=wtab)
    assert s.dtype == torch.float16 and s.shape == (N, 2 * proj.kp)
    x3 = P.mm2_project(s, num, aux, proj).cpu().numpy()
    num32, s32, aux32 = P.mm2_stream(N, T, 300, A, Vd, au, vi, ids32=ids32, table=table,
                                     wtab32=wtab, s_half=False)
    assert torch.equal(num32, num) and torch.equal(aux32, aux)
    f32 = P.mm2_project(s32, num32, aux32, proj).cpu().numpy()
    # the split is exact to fp16 hi + lo of the row-scaled fp32 sums
    sc = aux32[2][:, None]
    xs = s32 * sc
    hi = xs.half()
    assert torch.equal(s[:, :proj.kp], hi)
    assert torch.equal(s[:, proj.kp:], (xs - hi.float()).half())
    sw = np.where(ids >= 0, wt.astype(np.float32)[ids], 0).astype(np.float32)
    text = E[ids]
    ref = M.estimate_embedding_overall_gpu2(M.concat_inputs(text, audio, visual),
                                            M.params_from_module(gen.cpu()), sw, text)
    assert M.row_rel_err(x3, ref) < TOL
    assert M.row_rel_err(f32, ref) < TOL
    assert M.row_rel_err(x3, f32) < TOL


def test_fused_step_large_properties(gpu):
    """At 100k utterances x 40 frames x 3 x 300: unit rows, finite, deterministic."""
    N, T, V = 100_000, 40, 200_000
    inp = synth.device_workload(N, T, V, seed=9, device=gpu)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(gpu)
    step = P.FusedStep(inp, gen.networks())
    s1, m1 = [t.clone() for t in step.run()]
    s2, m2 = step.run()
    assert torch.equal(s1, s2) and torch.equal(m1, m2)
    assert torch.isfinite(m1).all() and torch.isfinite(s1).all()
    norms = torch.linalg.norm(m1.double(), dim=1)
    assert (norms - 1).abs().max().item() < 1e-5


@pytest.mark.parametrize("N", [1000, 129, 300])
def test_fused_pc_removal_matches_separate_kernel(gpu, N):
    """The bench order (Gram -> PC solve -> one projection kernel that also
    writes the PC-removed a2 rows, mmb_mm2_project_x3_rmpc) equals the
    separate mmb_pc_remove pass: MMB2 rows bit-identical, SIF rows to the
    fp64 dot's summation order; ragged last tiles (N % 128 != 0) included.
    Both against the CPU oracle of sif_functions.SIF_embedding too."""
    T, V = 40, 5000
    inp = synth.device_workload(N, T, V, A=300, Vd=300, seed=21, device=gpu)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(gpu)
    fused = P.FusedStep(inp, gen.networks(), stream_project=False, fork_projection=False)
    assert fused.fused_remove and fused.fork is None
    trace = {}
    s1, m1 = [t.clone() for t in fused.run(trace=trace)]
    assert "mm2_project+pc_remove" in trace and "pc_remove" not in trace
    sep = P.FusedStep(inp, gen.networks(), fuse_remove=False, stream_project=False)
    assert not sep.fused_remove
    s2, m2 = sep.run()
    torch.cuda.synchronize()
    assert torch.equal(m1, m2)
    assert M.row_rel_err(s1.cpu().numpy(), s2.cpu().numpy()) < 1e-6
    assert torch.equal(fused.pc, sep.pc)
    E = inp["table"].cpu().numpy()
    wt = inp["wtab"].cpu().numpy().astype(np.float64)
    ref = O.get_sentence_embeddings(E, wt, inp["ids"].cpu().numpy().astype(np.int64))
    assert M.row_rel_err(s1.cpu().numpy(), ref) < TOL


def test_chunked_overlapped_step_matches_single_chunk(gpu):
    """FusedStep(chunks=3): the stream kernel of chunk c+1 overlaps the projection
    and Gram of chunk c on a second HIP stream.  MMB2 rows are independent of the
    chunking (bit-identical); the SIF Gram is summed per chunk, so the PC-removed
    rows agree to fp64 summation order."""
    N, T, V = 5000, 24, 20_000
    inp = synth.device_workload(N, T, V, A=300, Vd=300, seed=11, device=gpu)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(gpu)
    one = P.FusedStep(inp, gen.networks(), chunks=1, stream_project=False)
    s1, m1 = [t.clone() for t in one.run()]
    three = P.FusedStep(inp, gen.networks(), chunks=3)
    assert len(three.bounds) == 3
    trace = {}
    s3, m3 = three.run(trace=trace)
    torch.cuda.synchronize()
    assert torch.equal(m1, m3)
    assert M.row_rel_err(s3.cpu().numpy(), s1.cpu().numpy()) < 1e-6
    assert len(trace["mm2_stream"]) == 3 and len(trace["mm2_project+gram"]) == 3
    with pytest.raises(ValueError):
        three.aux


@pytest.mark.parametrize("side_cus", [0, 96])
def test_overlapped_step_cu_masked_matches_single_chunk(gpu, side_cus):
    """The chunk pipeline (two-phase Gram, last chunk on every CU), with and
    without CU-masked side/main streams: MMB2 rows bit-identical to one
    chunk, SIF rows to fp64 summation order."""
    N, T, V = 6000, 40, 20_000
    inp = synth.device_workload(N, T, V, A=300, Vd=300, seed=12, device=gpu)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(gpu)
    one = P.FusedStep(inp, gen.networks(), chunks=1, stream_project=False)
    s1, m1 = [t.clone() for t in one.run()]
    four = P.FusedStep(inp, gen.networks(), chunks=4, side_cus=side_cus)
    assert len(four.bounds) == 4 and four.gram_parts
    for _ in range(2):  # a second step re-uses the buffers and the Gram partials
        s4, m4 = four.run()
    torch.cuda.synchronize()
    assert torch.equal(m1, m4)
    assert M.row_rel_err(s4.cpu().numpy(), s1.cpu().numpy()) < 1e-6


@pytest.mark.parametrize("N,T", [(3000, 40), (129, 40), (40, 300)])
def test_fused_step_int8_gram_vs_f64(gpu, N, T):
    """The default step's Gram (mmb_gram_i8 on the column bounds the stream
    kernel writes: wave kernel at T <= 64, workgroup kernel above) against the
    exact-f64 step: column bounds equal max |x|, G within 2e-9 relative, PC
    within 1e-9, MMB2 rows bit-identical, SIF rows to a few f32 ulps."""
    inp = synth.device_workload(N, T, 20_000, A=300, Vd=300, seed=51, device=gpu)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(gpu)
    a = P.FusedStep(inp, gen.networks(), gram_kind="i8")
    b = P.FusedStep(inp, gen.networks(), gram_kind="f64")
    assert a.gram_i8 and not b.gram_i8
    s1, m1 = [t.clone() for t in a.run()]
    s2, m2 = b.run()
    torch.cuda.synchronize()
    cm = a.colmax.cpu().numpy().view(np.float32)
    assert np.array_equal(cm, a.x.abs().amax(0).cpu().numpy())
    G1, G2 = a.G.cpu().numpy(), b.G.cpu().numpy()
    assert np.abs(G1 - G2).max() <= 2e-9 * np.abs(G2).max()
    assert np.abs(a.pc.cpu().numpy() - b.pc.cpu().numpy()).max() < 1e-9
    assert torch.equal(m1, m2)
    assert M.row_rel_err(s1.cpu().numpy(), s2.cpu().numpy()) < 2e-7  # f32 output ulps


def test_zero_weight_rows_sif_raises_mmb2_finite(gpu):
    """A row whose SIF weights are all zero: its a2 row is 0/0 = NaN (numpy,
    sif_functions.py:55) and the reference's TruncatedSVD rejects the split
    with a ValueError -- FusedStep.check() raises the same -- while its MMB2
    embedding is finite (the text term is 0, sif2.py:196-201) and every MMB2
    row matches the oracle."""
    from oracle import sif_oracle as O

    N, T, A, Vd, V = 600, 40, 300, 300, 5000
    torch.manual_seed(2)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None)
    E = synth.word_table(V, 300, seed=3)
    wt = synth.sif_weights(V, w0=0.0)
    ids = synth.token_ids(N, T, V, seed=4, ragged=True)
    ids[7] = 0  # all padding, weight 0
    audio = synth.frames(N, T, A, seed=5)
    visual = synth.frames(N, T, Vd, seed=6)
    inputs = {"table": torch.tensor(E, device=gpu),
              "wtab": torch.tensor(wt, device=gpu, dtype=torch.float32),
              "ids": torch.as_tensor(ids, dtype=torch.int32, device=gpu),
              "audio": torch.tensor(audio, device=gpu), "visual": torch.tensor(visual, device=gpu)}
    step = P.FusedStep(inputs, gen.to(gpu).networks())
    sif_out, mm2_out = [t.cpu().numpy() for t in step.run()]
    with pytest.raises(ValueError, match="NaN"):
        step.check()
    x = step.x.cpu().numpy()
    assert np.isnan(x[7]).all() and np.isfinite(np.delete(x, 7, 0)).all()
    sw = np.where(ids >= 0, wt.astype(np.float32)[ids], 0).astype(np.float32)
    text = E[ids]
    ref = M.estimate_embedding_overall_gpu2(M.concat_inputs(text, audio, visual),
                                            M.params_from_module(gen.cpu()), sw, text)
    assert np.isfinite(mm2_out).all()
    assert M.row_rel_err(mm2_out, ref) < TOL


def _pom_case(golden, case, n, A, Vd, seed):
    """Real POM transcript ids (pom_valid_ids 1089 / pom_test_ids 1357 wide,
    interior id-0 OOV tokens, trailing id-0 padding) + the real POM weights
    (w[0] = 1.0) from the g1 fixtures, the seeded V = 7763 table, and
    word-aligned U(-1, 1) frames set to -10 after each transcript's last token
    (the normalised pad value, utils.py:188-189)."""
    z = golden(case)
    ids = z["ids"][:n]
    N, T = ids.shape
    E = synth.word_table(int(z["V"]), 300, seed=int(z["table_seed"]))
    last = np.where(ids != 0, np.arange(T)[None, :], -1).max(1)
    pad = np.arange(T)[None, :] > last[:, None]
    audio = synth.frames(N, T, A, seed=seed)
    visual = synth.frames(N, T, Vd, seed=seed + 1)
    audio[pad] = -10.0
    visual[pad] = -10.0
    return E, z["weights"], ids, audio, visual


@pytest.mark.parametrize("case,n,A,Vd", [("g1_pom_valid", 32, 300, 300),
                                         ("g1_pom_test", 24, 300, 300),
                                         ("g1_pom_test", 48, 46, 37)])
def test_fused_step_pom_length_vs_oracle(gpu, golden, case, n, A, Vd):
    """BASELINE configs[2]: the bench step (SIF + PC removal + MMB2) at POM
    transcript length (T = 1089 / 1357 > the 512-token LDS chunk of the
    workgroup stream kernel, so the chunk loop wraps 3 times), against the
    oracle; 46 / 37-wide frames take the scalar-load variants."""
    E, wt, ids, audio, visual = _pom_case(golden, case, n, A, Vd, seed=40)
    N, T = ids.shape
    assert T > 1024
    torch.manual_seed(5)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None)
    inputs = {"table": torch.tensor(E, device=gpu),
              "wtab": torch.tensor(wt, device=gpu, dtype=torch.float32),
              "ids": torch.as_tensor(ids, dtype=torch.int32, device=gpu),
              "audio": torch.tensor(audio, device=gpu), "visual": torch.tensor(visual, device=gpu)}
    step = P.FusedStep(inputs, gen.to(gpu).networks())
    sif_out, mm2_out = step.run()
    step.check()
    ref_sif = O.get_sentence_embeddings(E, wt, ids)
    assert M.row_rel_err(sif_out.cpu().numpy(), ref_sif) < TOL
    sw = np.where(ids >= 0, wt.astype(np.float32)[ids], 0).astype(np.float32)
    text = E[ids]
    ref_mm2 = M.estimate_embedding_overall_gpu2(M.concat_inputs(text, audio, visual),
                                                 M.params_from_module(gen.cpu()), sw, text)
    assert M.row_rel_err(mm2_out.cpu().numpy(), ref_mm2) < TOL


@pytest.mark.parametrize("case,n,t_frames", [("g1_pom_test", 16, None), ("g1_pom_valid", 16, 160)])
def test_gpu2_drop_in_pom_length(gpu, golden, case, n, t_frames):
    """The sif2 drop-in at POM length through the --time_test call shape
    (simplesif.py:820-875): dense text / frames at T = 1357, and the POM form
    where the weighted text term runs over the unaligned transcript (L = 1089
    ids) while the frames are word-aligned with their own T = 160."""
    E, wt, ids, audio, visual = _pom_case(golden, case, n, 300, 300, seed=50)
    N, L_ = ids.shape
    T = t_frames or L_
    torch.manual_seed(6)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None)
    if t_frames:
        rng = np.random.default_rng(7)
        text = (E[rng.integers(1, E.shape[0], (N, T))]).astype(np.float32)
        audio, visual = audio[:, :T].copy(), visual[:, :T].copy()
    else:
        text = E[ids]
    emb = E[ids]
    sw = np.where(ids >= 0, wt.astype(np.float32)[ids], 0).astype(np.float32)
    t_ = lambda a: torch.tensor(a, device=gpu)
    au, vi, tx = t_(audio), t_(visual), t_(text)
    data = {"text": tx, "audio": au, "visual": vi, "audiovisual": torch.cat([au, vi], -1),
            "textaudio": torch.cat([tx, au], -1), "textvisual": torch.cat([tx, vi], -1),
            "textaudiovisual": torch.cat([tx, au, vi], -1)}
    masks = {k: None for k in data}
    g = gen.to(gpu)
    nets = {k: (g.embed2out[k]["mu"], g.embed2out[k]["log_sigma"]) for k in sif2.KEYS}
    with torch.no_grad():
        cs = sif2.estimate_embedding_overall_gpu2(data, masks, nets, t_(sw), t_(emb))
    ref = M.estimate_embedding_overall_gpu2(M.concat_inputs(text, audio, visual),
                                            M.params_from_module(gen.cpu()), sw, emb)
    assert M.row_rel_err(cs.cpu().numpy(), ref) < TOL


def test_gpu2_rejects_combinations_that_are_not_concatenations(gpu, golden):
    """The kernel streams text / audio / visual once; a combination tensor that
    is not their torch.cat (wrong width, wrong frames, or other contents)
    would give a different answer than the reference, so it raises."""
    z = golden("g4_mmb2_mosi")
    gen, E, ids, audio, visual, weights = _inputs(z, gpu)
    t_ = lambda a: torch.tensor(a, device=gpu)
    text, au, vi = t_(E[ids]), t_(audio), t_(visual)
    base = {"text": text, "audio": au, "visual": vi, "audiovisual": torch.cat([au, vi], -1),
            "textaudio": torch.cat([text, au], -1), "textvisual": torch.cat([text, vi], -1),
            "textaudiovisual": torch.cat([text, au, vi], -1)}
    masks = {k: None for k in base}
    g = gen.to(gpu)
    nets = {k: (g.embed2out[k]["mu"], g.embed2out[k]["log_sigma"]) for k in sif2.KEYS}
    sw = t_(np.where(ids >= 0, weights.astype(np.float32)[ids], 0).astype(np.float32))
    bad_width = dict(base, textvisual=torch.cat([text, vi[..., :-1]], -1))
    with pytest.raises(ValueError, match="textvisual.*features"):
        sif2.estimate_embedding_overall_gpu2(bad_width, masks, nets, sw, text)
    bad_frames = dict(base, audiovisual=base["audiovisual"][:, :-1])
    with pytest.raises(ValueError, match="audiovisual"):
        sif2.estimate_embedding_overall_gpu2(bad_frames, masks, nets, sw, text)
    other = dict(base, textaudio=torch.cat([text * 2, au], -1))
    with pytest.raises(ValueError, match="textaudio.*not data\\['text'\\]"):
        sif2.estimate_embedding_overall_gpu2(other, masks, nets, sw, text)
    with torch.no_grad():
        ok = sif2.estimate_embedding_overall_gpu2(base, masks, nets, sw, text)
    assert M.row_rel_err(ok.cpu().numpy(), z["cs_f64"]) < TOL


@pytest.mark.parametrize("T,V,A,Vd", [(40, 400_000, 300, 300), (20, 3016, 76, 48)],
                         ids=["configs3", "configs1_mosi"])
def test_full_size_step_sampled_rows_vs_oracle(gpu, T, V, A, Vd):
    """BASELINE configs[3] at full size (1M utterances x 40 x 3 x 300-d, V =
    400k, Zipf ids) and configs[1] at 1M utterances of MOSI shape (T = 20,
    COVAREP 76, FACET 48, V = 3016: the narrow fused kernel with the per-word
    text projection cache): the bench step itself, checked against the oracle where
    the check is size-independent.  MMB2 rows are per-utterance: 512 sampled
    rows against the oracle's sif2.estimate_embedding_overall_gpu2 on those
    rows (1e-5).  The SIF a2 rows of the sample against the oracle's
    get_weighted_average (2e-6), the step's PC (int8 Gram + device solve)
    against the oracle's randomized-SVD-from-Gram on the exact f64 Gram of
    all 1M a2 rows AND against the sklearn-path restatement
    (oracle.sif_oracle.compute_pc: LU-normalised power iteration on the 1M x
    300 f64 X itself) (1e-9), and the sample's PC-removed rows against the
    oracle's removal with that PC (1e-5)."""
    from oracle import sif_oracle as O

    N = 1_000_000
    inp = synth.device_workload(N, T, V, A=A, Vd=Vd, seed=1, device=gpu)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(gpu)
    step = P.FusedStep(inp, gen.networks())
    assert step.gram_i8 and step.stream_project == (A == 300)
    sif_out, mm2_out = step.run()
    step.check()
    torch.cuda.synchronize()
    rows = np.sort(np.random.default_rng(5).choice(N, 512, replace=False))
    ridx = torch.as_tensor(rows, device=gpu)
    E = inp["table"].cpu().numpy()
    wt = inp["wtab"].cpu().numpy()
    ids = inp["ids"][ridx].cpu().numpy().astype(np.int64)
    audio = inp["audio"][ridx].cpu().numpy()
    visual = inp["visual"][ridx].cpu().numpy()
    sw = wt[ids].astype(np.float32)
    text = E[ids]
    ref = M.estimate_embedding_overall_gpu2(M.concat_inputs(text, audio, visual),
                                            M.params_from_module(gen.cpu()), sw, text)
    assert M.row_rel_err(mm2_out[ridx].cpu().numpy(), ref) < TOL
    # a2 rows of the sample, then the PC over all rows from the exact Gram
    x_ref = O.get_weighted_average(E, ids, wt[ids].astype(np.float64))
    x = step.x.cpu().numpy()
    assert M.row_rel_err(x[rows], x_ref) < 2e-6
    X = x.astype(np.float64)
    G = X.T @ X
    # the reference algorithm itself on all 1M rows: TruncatedSVD(1, n_iter=7,
    # random_state=0)'s randomized SVD on X (sif_functions.py:58-67; the
    # restatement is pinned bit for bit to sklearn 1.7.2 by
    # test_oracle_golden.py), not only the device solver's CPU twin
    pc_sk = O.compute_pc(X, 1)
    del X
    z0 = np.random.RandomState(0).normal(size=(300, 11))
    pc = O.pc_from_gram(G, z0, 1, False)
    got = step.pc.cpu().numpy()
    assert np.abs(got - pc).max() < 1e-9
    assert np.abs(got - pc_sk).max() < 1e-9
    sif_ref = x_ref - (x_ref @ pc.T) @ pc
    assert M.row_rel_err(sif_out[ridx].cpu().numpy(), sif_ref) < TOL


def test_step_remerges_weights_only_after_an_update(gpu):
    """FusedStep re-merges the generator weights (mmb_mm2_prepare) only when a
    parameter changed in place since the last merge: a second step with the
    same weights skips it, an in-place update (what an optimiser step does)
    triggers it, and the rows then equal a fresh step's."""
    inp = synth.device_workload(700, 40, 5000, A=300, Vd=300, seed=61, device=gpu)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(gpu)
    step = P.FusedStep(inp, gen.networks())
    _, m1 = [t.clone() for t in step.run()]
    assert not step.proj.refresh_if_changed()
    with torch.no_grad():
        gen.embed2out["audio"]["mu"].weight.add_(0.05)
    assert step.proj.refresh_if_changed()
    with torch.no_grad():
        gen.embed2out["textvisual"]["log_sigma"].bias.mul_(0.9)
    _, m2 = [t.clone() for t in step.run()]
    _, m3 = P.FusedStep(inp, gen.networks()).run()
    torch.cuda.synchronize()
    assert not torch.equal(m1, m2)
    assert torch.equal(m2, m3)


@pytest.mark.parametrize("N,T,A,Vd", [(2048, 40, 300, 300), (1, 40, 300, 300), (15, 40, 300, 300),
                                     (17, 12, 300, 300), (700, 64, 300, 300), (5003, 40, 300, 300),
                                     (999, 33, 260, 292), (300, 40, 300, 256), (97, 40, 300, 20),
                                     (49, 40, 100, 300)])
def test_stream_project_matches_two_kernel_step(gpu, N, T, A, Vd):
    """The fused stream + projection kernel (mmb_mm2_stream_project: the sums
    s stay in an LDS ring, 48-row batches streamed modality by modality,
    partial last batch, narrow audio / visual widths)
    against the two-kernel step (mmb_mm2_stream -> HBM s -> mmb_mm2_project_x3):
    x, count and the column bounds bit-identical, the weight sum and MMB2 rows to f32
    rounding (per-piece scales, the same fp16 x3 products), PC-removed rows to
    the fp64 dot order -- and both against the CPU oracle."""
    from oracle import sif_oracle as O

    V = 20_000
    inp = synth.device_workload(N, T, V, A=A, Vd=Vd, seed=61, device=gpu)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(gpu)
    # the int8 Gram (its column bounds compared below) at every N
    a = P.FusedStep(inp, gen.networks(), stream_project=True, gram_kind="i8")
    # (the one-pass projection: the split-K one sums K in another f32 order,
    # tests/test_gpu_split.py)
    b = P.FusedStep(inp, gen.networks(), stream_project=False, gram_kind="i8",
                    split_projection=False)
    assert a.stream_project and a.s is None and not b.stream_project and b.proj_split is None
    trace = {}
    s1, m1 = [t.clone() for t in a.run(trace=trace)]
    assert "mm2_stream_project" in trace and "pc_remove" in trace
    s2, m2 = b.run()
    torch.cuda.synchronize()
    a.check()
    assert int(a.flag.item()) == 0
    # aux[2] is the text piece's scale in the fused kernel (the whole row's
    # before); its weight sum is a 64-lane f32 sum in another order (DPP rows)
    assert torch.equal(a.x, b.x) and torch.equal(a.aux[0], b.aux[0])
    assert torch.allclose(a.aux[1], b.aux[1], rtol=1e-6, atol=0)
    assert torch.equal(a.colmax, b.colmax)
    assert M.row_rel_err(m1.cpu().numpy(), m2.cpu().numpy()) < 1e-6
    assert torch.equal(a.pc, b.pc)
    # SIF rows to the fp64 dot order, relative to the a2 rows (N = 1 removes
    # the whole row: x - (x . pc) pc is ~1e-14 of x)
    xmax = a.x.abs().max().item()
    assert (s1 - s2).abs().max().item() <= 1e-6 * xmax
    E = inp["table"].cpu().numpy()
    wt = inp["wtab"].cpu().numpy().astype(np.float64)
    ids = inp["ids"].cpu().numpy().astype(np.int64)
    if N > 1:
        ref_sif = O.get_sentence_embeddings(E, wt, ids)
        assert M.row_rel_err(s1.cpu().numpy(), ref_sif) < TOL
    if N == 1:  # the reference's gpu2 cannot take one utterance (squeeze, sif2.py:200-207)
        return
    audio, visual = inp["audio"].cpu().numpy(), inp["visual"].cpu().numpy()
    sw = np.where(ids >= 0, wt.astype(np.float32)[ids], 0).astype(np.float32)
    text = E[ids]
    ref_mm2 = M.estimate_embedding_overall_gpu2(M.concat_inputs(text, audio, visual),
                                                 M.params_from_module(gen.cpu()), sw, text)
    assert M.row_rel_err(m1.cpu().numpy(), ref_mm2) < TOL


def test_stream_project_repeatable_and_unit_rows(gpu):
    """Bench-like size (60k utterances, V = 400k Zipf ids): two steps of the
    fused kernel are bit-identical (the ring hand-over is order-independent),
    rows are unit length, no hand-over timed out."""
    inp = synth.device_workload(60_000, 40, 400_000, seed=62, device=gpu)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(gpu)
    step = P.FusedStep(inp, gen.networks())
    assert step.stream_project
    s1, m1 = [t.clone() for t in step.run()]
    s2, m2 = step.run()
    torch.cuda.synchronize()
    step.check()
    assert torch.equal(s1, s2) and torch.equal(m1, m2)
    norms = torch.linalg.norm(m1.double(), dim=1)
    assert (norms - 1).abs().max().item() < 1e-5


def test_default_step_at_mosi_widths_is_narrow_fused(gpu):
    """configs[1] frame widths (COVAREP 76, FACET 48, V = 3016): FusedStep's
    default is the narrow fused kernel (r04; the wide-frame fused kernel does
    not pay here, pipeline.fused_pays), its rows within the bar of the CPU
    oracle (SIF) and of the reference's gpu2 restatement (MMB2)."""
    from oracle import sif_oracle as O

    N, T, A, Vd, V = 3000, 20, 76, 48, 3016
    inp = synth.device_workload(N, T, V, A=A, Vd=Vd, seed=63, device=gpu)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(gpu)
    step = P.FusedStep(inp, gen.networks())
    assert not step.stream_project and step.narrow_fused and step.s is None
    trace = {}
    s1, m1 = step.run(trace=trace, check=True)
    assert "mm2_stream_project_narrow" in trace and "mm2_stream" not in trace
    E = inp["table"].cpu().numpy()
    wt = inp["wtab"].cpu().numpy().astype(np.float64)
    ids = inp["ids"].cpu().numpy().astype(np.int64)
    assert M.row_rel_err(s1.cpu().numpy(), O.get_sentence_embeddings(E, wt, ids)) < TOL
    audio, visual = inp["audio"].cpu().numpy(), inp["visual"].cpu().numpy()
    sw = np.where(ids >= 0, wt.astype(np.float32)[ids], 0).astype(np.float32)
    ref = M.estimate_embedding_overall_gpu2(M.concat_inputs(E[ids], audio, visual),
                                            M.params_from_module(gen.cpu()), sw, E[ids])
    assert M.row_rel_err(m1.cpu().numpy(), ref) < TOL


@pytest.mark.parametrize("N,T,A,Vd,V", [(3000, 20, 76, 48, 3016), (1001, 40, 76, 48, 3016),
                                        (517, 64, 128, 100, 5000), (64, 7, 20, 8, 300),
                                        (259, 33, 44, 124, 400_000), (5, 1, 76, 48, 3016)])
def test_narrow_frame_stream_kernel(gpu, N, T, A, Vd, V):
    """The narrow-frame stream kernel (utt_narrow_kernel: frame rows of <= 32
    float4 units packed 2-32 rows per wave-instruction, every frame load of an
    utterance issued at once; fp16 s) against utt_wave_kernel (the fp32-s
    stream of the same inputs): the text sums are the same operations in the
    same order, so x, count, weight sum and the column bounds are
    bit-identical; the frame sums (per-slot partials added slot by slot) and
    the dequantised fp16 hi + lo text sums equal the fp32 sums to f32
    rounding.
    Ragged ids with negative (wrapping) and out-of-range ids (flagged) mixed
    in; T past one issue group (40, 64 frames: later groups after the text)."""
    rng = np.random.default_rng(N)
    inp = synth.device_workload(N, T, V, A=A, Vd=Vd, seed=70 + T, device=gpu)
    ids = inp["ids"].clone()
    if N > 10:
        r = torch.as_tensor(rng.integers(0, N, 5), device=gpu)
        ids[r, 0] = -3  # wraps to V - 3, like numpy fancy indexing
    table, wtab = inp["table"], inp["wtab"]
    proj = P.MMB2Projection(models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(gpu).networks(),
                            300, A, Vd, T, gpu)
    f1 = torch.zeros(1, dtype=torch.int32, device=gpu)
    f2 = torch.zeros(1, dtype=torch.int32, device=gpu)
    cm1 = torch.zeros(300, dtype=torch.int32, device=gpu)
    cm2 = torch.zeros(300, dtype=torch.int32, device=gpu)
    nb = L.query("mmb_mm2_colmax_ws_bytes", 300)
    ws1 = torch.empty((nb + 15) // 16 * 16, dtype=torch.uint8, device=gpu)
    ws2 = torch.empty_like(ws1)
    num, s, aux = P.mm2_stream(N, T, 300, A, Vd, inp["audio"], inp["visual"], ids32=ids, table=table,
                               wtab32=wtab, flag=f1, colmax=cm1, colmax_ws=ws1)
    num32, s32, aux32 = P.mm2_stream(N, T, 300, A, Vd, inp["audio"], inp["visual"], ids32=ids,
                                     table=table, wtab32=wtab, s_half=False, flag=f2, colmax=cm2,
                                     colmax_ws=ws2)
    torch.cuda.synchronize()
    assert s.dtype == torch.float16 and s.shape == (N, 2 * proj.kp)
    assert torch.equal(num, num32) and torch.equal(aux[:2], aux32[:2])
    assert torch.equal(cm1, cm2) and int(f1.item()) == int(f2.item()) == 0
    k = 2 * (300 + A + Vd)
    deq = (s[:, :k].double() + s[:, proj.kp:proj.kp + k].double()) / aux[2][:, None].double()
    ref = s32[:, :k].double()
    err = (deq - ref).abs().amax(1) / ref.abs().amax(1).clamp_min(1e-30)
    assert err.max().item() < 2e-6
    assert (s[:, k:proj.kp] == 0).all() and (s[:, proj.kp + k:] == 0).all()
    # the row scale is the power of 2 of the row max: equal but where the max
    # sits within rounding of a power of two
    assert (aux[2] == aux32[2]).float().mean().item() > 0.99
    # an out-of-range id: flagged, the row contributes nothing (as in the wave kernel)
    bad = ids.clone()
    bad[N // 2, 0] = V + 7
    f3 = torch.zeros(1, dtype=torch.int32, device=gpu)
    n3, _, a3 = P.mm2_stream(N, T, 300, A, Vd, inp["audio"], inp["visual"], ids32=bad, table=table,
                             wtab32=wtab, flag=f3)
    f4 = torch.zeros(1, dtype=torch.int32, device=gpu)
    n4, _, a4 = P.mm2_stream(N, T, 300, A, Vd, inp["audio"], inp["visual"], ids32=bad, table=table,
                             wtab32=wtab, s_half=False, flag=f4)
    torch.cuda.synchronize()
    assert int(f3.item()) == int(f4.item()) and int(f3.item()) & L.MMB_FLAG_ID_RANGE
    # (an utterance left with no valid token is 0 / 0 = NaN in both, as in numpy)
    assert torch.allclose(n3, n4, rtol=0, atol=0, equal_nan=True) and torch.equal(a3[:2], a4[:2])


def _split_check(gen, sp, sif_out, mm2_out, pc, rows, x, ref_rows=None, ref_pc=None):
    """One split against the oracle: SIF over the whole split (its own PC,
    the reference's loops + sklearn-path randomized SVD), MMB2 on a row sample.

    PC bars: the sklearn-path restatement run on the step's own a2 rows x
    (f64) pins the device solve to 1e-12; against the PC of the reference's
    rows the bar is 1e-7 -- the a2 rows are f32 sums of up to 1357 weighted
    table rows, and the device's summation order moves them by ~1e-7 of their
    scale (row-relative 2e-6 bar elsewhere), which moves the PC by ~2e-8 on
    the real POM valid split (s1/s2 = 24)."""
    E, wt, ids = sp["table"], sp["weights"], sp["ids"]
    sif_ref = O.get_sentence_embeddings(E, wt, ids)
    sif = sif_out.double().cpu().numpy()
    # SIF rows: 1e-5 row-relative of the reference's f32 path -- or, where the
    # transcripts are long (POM: up to 1357 tokens, the a2 rows f32 sums of
    # ~370 table rows before a PC removal that cancels ~95 % of them), within
    # 3x the reference's OWN distance from the exact (f64) evaluation: two f32
    # summation orders of the same rows then differ by about that much
    exact = O.get_sentence_embeddings(E.astype(np.float64), wt, ids)
    e_ref, e_gpu = M.row_rel_err(sif_ref, exact), M.row_rel_err(sif, exact)
    print(f"SIF row-rel: gpu vs reference {M.row_rel_err(sif, sif_ref):.2e}, gpu vs exact "
          f"{e_gpu:.2e}, reference vs exact {e_ref:.2e}")
    assert M.row_rel_err(sif, sif_ref) < TOL or e_gpu <= 3 * e_ref
    got = pc.cpu().numpy()
    assert np.abs(got - O.compute_pc(x.double().cpu().numpy())).max() < 1e-12
    pc_ref = O.compute_pc(O.get_weighted_average(E, ids, O.seq2weight(ids, np.ones(ids.shape), wt)))
    assert np.abs(got - pc_ref).max() < 1e-7
    if ref_pc is not None:  # the reference's own run (g11)
        assert np.abs(got - ref_pc).max() < 1e-7
        assert np.array_equal(sif_ref[::8], ref_rows)  # the oracle IS the reference here
    r = rows
    sw = O.seq2weight(ids[r], np.ones(ids[r].shape), wt)
    text = E[ids[r]]
    ref = M.estimate_embedding_overall_gpu2(M.concat_inputs(text, sp["audio"][r], sp["visual"][r]),
                                            M.params_from_module(gen), sw, text)
    assert M.row_rel_err(mm2_out[torch.as_tensor(r, device=mm2_out.device)].cpu().numpy(),
                         ref) < TOL


@pytest.mark.parametrize("mode", ["eager", "graph"])
def test_real_pom_splits_vs_reference_and_oracle(gpu, golden, mode):
    """configs[2] at its real call pattern: the reference's own pom_valid_ids
    (100 x 1089) and pom_test_ids (203 x 1357) with pom_word_weights.npy, SIF
    + MMB2 once per split, each split with its own PC (simplesif.py:296-311;
    n < 300: sklearn's transposed branch).  SIF rows and PC against the
    reference's recorded run (g11) and the oracle, MMB2 on 32 rows per split
    against the oracle's sif2.estimate_embedding_overall_gpu2; the graph mode
    (both splits in ONE HIP graph, concurrent branches) equals eager bit for bit."""
    z = golden("g11_pom_splits")
    splits = synth.pom_splits(z["valid_ids"], z["test_ids"], z["weights"], int(z["table_seed"]))
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 300, 300, norm=None).to(gpu)
    steps = [P.FusedStep(synth.to_device(sp, gpu), gen.networks()) for sp in splits]
    eager = [[t.clone() for t in st.run(check=True)] for st in steps]
    if mode == "graph":
        g = P.StepGraph(steps, concurrent=True)
        for _ in range(2):
            outs = g.run(check=True)
        for (s0, m0), (s1, m1) in zip(eager, outs):
            assert torch.equal(s0, s1) and torch.equal(m0, m1)
    gen_cpu = gen.cpu()
    for nm, sp, st, (sif_out, mm2_out) in zip(("valid", "test"), splits, steps, eager):
        rows = np.sort(np.random.default_rng(7).choice(sp["ids"].shape[0], 32, replace=False))
        _split_check(gen_cpu, sp, sif_out, mm2_out, st.pc, rows, st.x, z[f"{nm}_out_rows"],
                     z[f"{nm}_pc"])


def test_mosi_splits_each_with_its_own_pc(gpu):
    """configs[0]/[1] at their real call pattern: three MOSI-shaped splits
    (1284 / 229 / 686 utterances, T = 20, A = 76, Vd = 48; 229 < 300 takes
    the transposed branch) in one concurrent HIP graph: every split's SIF rows
    and PC against the oracle, MMB2 on 64 rows per split."""
    splits = synth.mosi_splits()
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 76, 48, norm=None).to(gpu)
    steps = [P.FusedStep(synth.to_device(sp, gpu), gen.networks()) for sp in splits]
    outs = P.StepGraph(steps, concurrent=True).run(check=True)
    gen_cpu = gen.cpu()
    for sp, st, (sif_out, mm2_out) in zip(splits, steps, outs):
        rows = np.sort(np.random.default_rng(8).choice(sp["ids"].shape[0], 64, replace=False))
        _split_check(gen_cpu, sp, sif_out, mm2_out, st.pc, rows, st.x)


def test_step_graph_follows_weight_updates(gpu):
    """A captured step re-merges the generator weights eagerly before the
    replay when a parameter changed in place (what an optimiser step does):
    the replayed rows equal a fresh eager step's."""
    inp = synth.device_workload(1500, 20, 3016, A=76, Vd=48, seed=71, device=gpu)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, 76, 48, norm=None).to(gpu)
    st = P.FusedStep(inp, gen.networks())
    g = P.StepGraph(st)
    s0, m0 = [t.clone() for t in g.run(check=True)]
    with torch.no_grad():
        gen.embed2out["visual"]["mu"].weight.mul_(1.5)
    s1, m1 = [t.clone() for t in g.run(check=True)]
    fresh = P.FusedStep(inp, gen.networks())
    s2, m2 = fresh.run(check=True)
    assert torch.equal(s1, s2) and torch.equal(m1, m2) and not torch.equal(m0, m1)
    assert torch.equal(s0, s1)


@pytest.mark.parametrize("N,T,A,Vd,V", [(3000, 20, 76, 48, 3016), (1, 20, 76, 48, 3016),
                                        (31, 20, 76, 48, 3016), (1001, 40, 76, 48, 3016),
                                        (517, 64, 64, 56, 5000), (64, 7, 20, 8, 300),
                                        (259, 33, 44, 76, 16384), (5, 1, 76, 48, 3016),
                                        (6000, 20, 76, 48, 3016),
                                        (77, 20, 76, 48, 17)])
def test_narrow_fused_matches_two_kernel_step(gpu, N, T, A, Vd, V):
    """The narrow fused kernel (mmb_mm2_stream_project_narrow: per-word text
    projection from the text cache, hot words from LDS, 32-utterance batches,
    the audio / visual GEMM in-launch) against the two-kernel narrow step
    (utt_narrow_kernel -> HBM s -> mmb_mm2_project_x3) on the same inputs:
    count identical, weight sum and x to f32 rounding (the fused kernel sums
    an utterance's hot words first, then its cold words; its weight sum by
    DPP rows); the PC equal to
    the sklearn-path restatement's on the fused step's own x; the MMB2 rows
    to f32 rounding (another grouping of the same closed form) and both
    within the bar of the CPU oracle.  Partial and single-row batches,
    T from 1 to 64, frame widths 8-128, fewer words than LDS slots (V = 17),
    the largest cached vocabulary (16384), wrapped negative ids; 1, 2 and 4
    utterances per wave and batch (N below ~4k, ~4-8k, larger).  (Wider
    frames -- kq(A) + kq(Vd) > 256 -- and larger vocabularies keep the
    two-kernel step: narrow_fused_supported.)"""
    from oracle import sif_oracle as O

    assert not P.narrow_fused_supported(T, 300, 128, 100, V)
    assert not P.narrow_fused_supported(T, 300, A, Vd, 16385)

    rng = np.random.default_rng(N + T)
    inp = synth.device_workload(N, T, V, A=A, Vd=Vd, seed=90 + T, device=gpu)
    if N > 10:
        r = torch.as_tensor(rng.integers(0, N, 5), device=gpu)
        inp["ids"][r, 0] = -3  # wraps to V - 3, like numpy fancy indexing
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(gpu)
    a = P.FusedStep(inp, gen.networks(), narrow_fused=True)
    b = P.FusedStep(inp, gen.networks(), narrow_fused=False)
    assert a.narrow_fused and not b.narrow_fused and a.gram_i8 == b.gram_i8
    s1, m1 = [t.clone() for t in a.run()]
    s2, m2 = b.run()
    torch.cuda.synchronize()
    assert int(a.flag.item()) == int(b.flag.item()) == 0
    # count exact; the weight sum is a 64-lane f32 sum in another order (DPP rows)
    assert torch.equal(a.aux[0], b.aux[0])
    assert torch.allclose(a.aux[1], b.aux[1], rtol=1e-6, atol=0)
    assert M.row_rel_err(a.x.cpu().numpy(), b.x.cpu().numpy()) < 2e-6
    if N >= 300:  # sklearn's direct randomized-SVD branch
        pc_sk = O.compute_pc(a.x.double().cpu().numpy())
        assert np.abs(a.pc.cpu().numpy() - pc_sk).max() < 1e-10
    assert M.row_rel_err(m1.cpu().numpy(), m2.cpu().numpy()) < 2e-6
    xmax = a.x.abs().max().item()
    assert (s1 - s2).abs().max().item() <= 1e-6 * xmax
    norms = torch.linalg.norm(m1.double(), dim=1)
    assert (norms - 1).abs().max().item() < 1e-5
    if N == 1:
        return
    E = inp["table"].cpu().numpy()
    wt = inp["wtab"].cpu().numpy().astype(np.float64)
    ids = inp["ids"].cpu().numpy().astype(np.int64)
    rows = np.sort(rng.choice(N, min(N, 256), replace=False))
    assert M.row_rel_err(s1.cpu().numpy(), O.get_sentence_embeddings(E, wt, ids)) < TOL
    audio, visual = inp["audio"].cpu().numpy()[rows], inp["visual"].cpu().numpy()[rows]
    idr = ids[rows]
    sw = np.where(idr >= 0, wt.astype(np.float32)[idr], 0).astype(np.float32)
    ref = M.estimate_embedding_overall_gpu2(M.concat_inputs(E[idr], audio, visual),
                                            M.params_from_module(gen.cpu()), sw, E[idr])
    assert M.row_rel_err(m1.cpu().numpy()[rows], ref) < TOL


def test_narrow_fused_column_bounds_flags_and_weight_updates(gpu):
    """The narrow fused kernel's column bounds (mmb_gram_i8's input) are the
    column maxima of its own x (mmb_colmax), its Gram the int8 Gram of that x;
    an out-of-range id is flagged (IndexError from
    check()); a zero-weight utterance raises ValueError like the reference; a
    generator update re-merges Wm AND rebuilds the text cache (the replayed
    rows equal a fresh step's)."""
    N, T, A, Vd, V = 40_000, 20, 76, 48, 3016
    inp = synth.device_workload(N, T, V, A=A, Vd=Vd, seed=95, device=gpu)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(gpu)
    a = P.FusedStep(inp, gen.networks(), narrow_fused=True)
    b = P.FusedStep(inp, gen.networks(), narrow_fused=False)
    assert a.gram_i8 and b.gram_i8
    a.run(check=True)
    b.run(check=True)
    torch.cuda.synchronize()
    assert torch.equal(a.colmax, P.colmax(a.x)) and torch.equal(a.G, P.gram_i8(a.x, a.colmax))
    assert M.row_rel_err(a.x.cpu().numpy(), b.x.cpu().numpy()) < 2e-6
    with torch.no_grad():
        gen.embed2out["textaudio"]["mu"].weight.mul_(1.25)
    _, m1 = [t.clone() for t in a.run(check=True)]
    _, m2 = P.FusedStep(inp, gen.networks(), narrow_fused=True).run(check=True)
    assert torch.equal(m1, m2)
    bad = {k: v.clone() if k == "ids" else v for k, v in inp.items()}
    bad["ids"][7, 3] = V + 5
    with pytest.raises(IndexError):
        P.FusedStep(bad, gen.networks(), narrow_fused=True).run(check=True)
    zw = {k: v.clone() if k in ("ids", "wtab") else v for k, v in inp.items()}
    zw["wtab"][zw["ids"][11]] = 0.0  # every token of utterance 11 now weighs 0
    with pytest.raises(ValueError):
        P.FusedStep(zw, gen.networks(), narrow_fused=True).run(check=True)
