"""CPU: host-side logic of the drop-in (no GPU needed)."""
import numpy as np
import pytest
import torch
from torch.utils.data import DataLoader

import models
import sentiment_model as SM


def test_mmb2_parameter_layout_and_init_order():
    torch.manual_seed(0)
    g = models.AudioVisualGeneratorMultimodal(300, 76, 48, norm=None)
    assert list(g.embed2out.keys()) == list(models.MMB2_KEYS)
    widths = {k: g.embed2out[k]["mu"].weight.shape[0] for k in models.MMB2_KEYS}
    assert widths == {"audio": 76, "visual": 48, "audiovisual": 124, "textaudio": 376,
                      "textvisual": 348, "textaudiovisual": 424}
    assert all(g.embed2out[k]["mu"].weight.shape[1] == 300 for k in models.MMB2_KEYS)
    g1 = models.AudioVisualGeneratorMultimodal(300, 76, 48, unimodal=True)
    assert list(g1.embed2out.keys()) == ["audio", "visual"]


def test_combo_segments_follow_cat_order():
    assert models.combo_dims("textaudiovisual", 300, 76, 48) == [("text", 300), ("audio", 76),
                                                                   ("visual", 48)]
    assert models.combo_dims("audiovisual", 300, 76, 48) == [("audio", 76), ("visual", 48)]


@pytest.mark.parametrize("n,bs", [(1284, 32), (229, 32), (33, 32), (5, 32)])
def test_loader_emulation_consumes_rng_like_iteration(n, bs):
    data = SM.SentimentData(np.arange(n, dtype=np.float32), torch.device("cpu"))
    loader = DataLoader(data, batch_size=bs, shuffle=True)
    torch.manual_seed(7)
    real = [[j.clone() for j, _ in loader] for _ in range(3)]
    after_real = torch.rand(4)
    torch.manual_seed(7)
    emu = [SM._epoch_batches(loader) for _ in range(3)]
    after_emu = torch.rand(4)
    assert torch.equal(after_real, after_emu)
    for r, e in zip(real, emu):
        assert len(r) == len(e)
        for a, b in zip(r, e):
            assert torch.equal(a, b)


@pytest.mark.parametrize("n,bs,shuffle", [(1284, 32, True), (229, 32, True), (5, 32, True),
                                          (33, 32, False)])
def test_epoch_perm_consumes_rng_like_iteration(n, bs, shuffle):
    """_epoch_perm (one randperm per pass, the fast path of the one-launch
    training loop) yields the rows of real DataLoader iteration in order and
    leaves the global RNG where iteration leaves it -- interleaved with a
    second loader, as the reference's train / validation passes are."""
    data = SM.SentimentData(np.arange(n, dtype=np.float32), torch.device("cpu"))
    loader = DataLoader(data, batch_size=bs, shuffle=shuffle)
    other = DataLoader(SM.SentimentData(np.arange(7, dtype=np.float32), torch.device("cpu")),
                       batch_size=bs, shuffle=True)
    torch.manual_seed(11)
    real = []
    for _ in range(3):
        real.append(torch.cat([j.clone() for j, _ in loader]))
        real.append(torch.cat([j.clone() for j, _ in other]))
    after_real = torch.rand(4)
    torch.manual_seed(11)
    emu = []
    for _ in range(3):
        emu.append(SM._epoch_perm(loader))
        emu.append(SM._epoch_perm(other))
    after_emu = torch.rand(4)
    assert torch.equal(after_real, after_emu)
    for r, e in zip(real, emu):
        assert torch.equal(r, e)


def test_f32_epoch_mean_matches_tensor_arithmetic():
    vals = np.random.default_rng(0).random(41).astype(np.float32)
    acc = 0
    for v in vals:
        acc = acc + torch.tensor(v)
    ref = float(acc / 41)
    assert SM._f32_mean_of(vals, 41) == ref


def test_sentiment_model_init_matches_reference_order():
    torch.manual_seed(3)
    m = SM.SentimentModel(300, 100, 1)
    torch.manual_seed(3)
    h = torch.nn.Linear(300, 100)
    o = torch.nn.Linear(100, 1)
    assert torch.equal(m.hidden1.weight, h.weight) and torch.equal(m.out.bias, o.bias)


def test_side_cu_sets_are_balanced_and_disjoint():
    """The overlapped step's side CU set (pipeline.side_cu_set): the requested
    count, evenly spread over the 8 residues mod 8 and the 8 blocks of 32 mask
    bits (either way the driver may deal bits to XCDs) for the balanced
    layout."""
    import collections

    import pipeline as P

    for side in (64, 80, 96, 112, 128):
        s = P.side_cu_set(256, side, "balanced")
        assert len(s) == side and len(set(s)) == side and max(s) < 256
        assert set(collections.Counter(c % 8 for c in s).values()) == {side // 8}
        assert set(collections.Counter(c // 32 for c in s).values()) == {side // 8}
        assert len(P.side_cu_set(256, side, "high")) == side
        assert len(P.side_cu_set(256, side, "strided")) == side


def _mm_data(n=4, t=6, d=8, a=5, vd=3, seed=0):
    g = torch.Generator().manual_seed(seed)
    tx, au, vi = (torch.randn(n, t, f, generator=g) for f in (d, a, vd))
    return {"text": tx, "audio": au, "visual": vi, "audiovisual": torch.cat([au, vi], -1),
            "textaudio": torch.cat([tx, au], -1), "textvisual": torch.cat([tx, vi], -1),
            "textaudiovisual": torch.cat([tx, au, vi], -1)}


def test_gpu2_combination_check_accepts_concatenations_and_names_the_bad_key():
    """sif2.check_combinations (host side of the gpu2 drop-in): concatenations
    pass; a wrong width, a wrong frame count, or other contents raise a
    ValueError naming the key (simplesif.py:825-830 builds them with torch.cat)."""
    import sif2

    d = _mm_data()
    sif2.check_combinations(d)
    nan = _mm_data()
    nan["audio"][0, 0, 0] = float("nan")
    nan["audiovisual"] = torch.cat([nan["audio"], nan["visual"]], -1)
    nan["textaudio"] = torch.cat([nan["text"], nan["audio"]], -1)
    nan["textaudiovisual"] = torch.cat([nan["text"], nan["audio"], nan["visual"]], -1)
    sif2.check_combinations(nan)  # NaN frames are still the same concatenation
    bad = dict(d, textaudiovisual=d["textaudiovisual"][..., :-1])
    with pytest.raises(ValueError, match="textaudiovisual.*8 \\+ 5 \\+ 3"):
        sif2.check_combinations(bad)
    bad = dict(d, textvisual=d["textvisual"][:, :-1])
    with pytest.raises(ValueError, match="textvisual"):
        sif2.check_combinations(bad)
    swapped = dict(d, audiovisual=torch.cat([d["visual"], d["audio"]], -1))
    with pytest.raises(ValueError, match="audiovisual"):
        sif2.check_combinations(swapped)
    sif2.CHECK_CONCATENATIONS = False
    try:
        sif2.check_combinations(dict(d, textaudio=d["textaudio"] * 2))  # widths only
    finally:
        sif2.CHECK_CONCATENATIONS = True


def test_npc_limit_is_a_clear_value_error():
    import pipeline as P

    for npc in range(1, 7):
        P.check_npc(npc)
    for npc in (0, 7, 20):
        with pytest.raises(ValueError, match="npc"):
            P.check_npc(npc)


def test_tiny_splits_pc_restatement_matches_sklearn():
    """The device solver's math (Gram-only randomized SVD, pc_from_gram via
    CPUOps) equals scikit-learn's TruncatedSVD also for splits smaller than
    the npc + 10 block (the rank-deficient LU branch)."""
    from sklearn.decomposition import TruncatedSVD

    import pipeline as P
    from oracle import sif_oracle as O

    for n in (1, 2, 5, 10, 11):
        rng = np.random.default_rng(n)
        g = rng.standard_normal(300)
        X = (0.4 * rng.standard_normal((n, 300)) + 0.3 * g).astype(np.float32)
        svd = TruncatedSVD(n_components=1, n_iter=7, random_state=0)
        with np.errstate(all="ignore"):
            ref = svd.fit(X.astype(np.float64)).components_
        pc = P.global_pc(torch.from_numpy(X), None, 1, n, 0, None, ops=O.CPUOps).numpy()
        assert np.abs(pc - ref).max() < 1e-12
        assert np.abs(O.compute_pc(X.astype(np.float64), 1) - ref).max() < 1e-14


def test_fused_step_dispatch_by_frame_width():
    """FusedStep's default kernel choice (pipeline.fused_pays): the fused
    stream + projection kernel for wide frame rows (configs[3]: 300 / 300),
    the two-kernel step for MOSI's narrow ones (76 / 48), where it measured
    1.5x faster."""
    import pipeline as P

    assert P.fused_pays(300, 300) and P.fused_pays(256, 512)
    assert not P.fused_pays(76, 48) and not P.fused_pays(300, 48) and not P.fused_pays(255, 300)


def test_word_weights_file_and_mosi_table(tmp_path, monkeypatch, capsys):
    """sif.py:14-76: a / (a + count / total) per word; malformed lines echoed and
    skipped; the MOSI table by lower-cased lookup, unknown words 1.0, unmapped
    indices 0, cached to word_weights.npy."""
    import sif

    f = tmp_path / "freq.txt"
    f.write_text("the 600\n\nof 300\nbad line here\ncat 100\n")
    ww = sif.get_word_weights(str(f), a=1e-3)
    assert capsys.readouterr().out.strip() == "['bad', 'line', 'here']"
    assert ww == {w: 1e-3 / (1e-3 + c / 1000.0) for w, c in (("the", 600.0), ("of", 300.0), ("cat", 100.0))}
    monkeypatch.chdir(tmp_path)
    with pytest.raises(NameError):
        sif.load_mosi_weights()
    tab = sif.load_mosi_weights({"The": 1, "dog": 2, "CAT": 4}, word_freq_file=str(f))
    np.testing.assert_array_equal(tab, [0.0, ww["the"], 1.0, 0.0, ww["cat"]])
    assert "# of words with unknown weight 1" in capsys.readouterr().out
    np.testing.assert_array_equal(sif.load_mosi_weights(), tab)  # the cached table


def test_check_step_sigma_block_form(capsys):
    """simplesif.check_step with the whole-block sigma minimum (sigma_mins on
    the fused generator head's column views): 'boo!' printed for exactly the
    keys whose own sigma minimum is below 1e-7 (read from `out` only then),
    nothing otherwise; the per-key form gives the same prints."""
    import simplesif

    blk = torch.full((4, 6), 0.5)
    views = blk.split([2, 1, 3], dim=1)
    out = {k: {"mu": torch.zeros_like(v), "sigma": v} for k, v in zip(("audio", "visual", "audiovisual"), views)}
    rest = torch.tensor([0.0, 1.0, 2.0, 3.0])  # word min, three Gaussian mins (finite)
    loss = torch.tensor([7.0])
    sig = simplesif.sigma_mins(out)
    assert sig.shape == (1,)
    vals = torch.cat([loss, sig, rest])
    assert simplesif.check_step(out, vals, (4, 300), len(vals) - 2 - len(out)) == 7.0
    assert "boo!" not in capsys.readouterr().out
    blk[2, 3] = 1e-9  # column 3: the third key
    sig = simplesif.sigma_mins(out)
    simplesif.check_step(out, torch.cat([loss, sig, rest]), (4, 300), 1)
    text = capsys.readouterr().out
    assert text.count("boo!") == 1 and "1.0000e-09" in text  # the third key's dict
    per_key = torch.stack([d["sigma"].min() for d in out.values()]).abs()
    simplesif.check_step(out, torch.cat([loss, per_key, rest]), (4, 300))
    assert capsys.readouterr().out == text
