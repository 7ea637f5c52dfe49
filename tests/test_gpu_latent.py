"""GPU: the latent-objective kernels (csrc/latent_kernels.hip via latent.py /
losses.py) and the simplesif.py CLI against the reference's own outputs
(tests/golden/g7_*, g8_matrix, g9_cli_*) and the CPU oracle.

Tolerances (fp32 arithmetic on both sides, different summation order):
  log-likelihoods   |y - y_ref| <= 2e-5 |y_ref| + 1e-4
  gradients         per row, max|g - g_ref| <= 2e-4 max|g_ref|
  CLI run           pre/embed.bin (SIF) row-relative 1e-5; post/embed.bin
                    row-relative 1e-3 after the optimisation epochs; loss
                    files 1e-4 relative; regressor MAE 1e-3 relative.
"""
import copy
import json
import os

import numpy as np
import pytest
import torch

import synth
from oracle import latent_oracle as LO

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def close(y, ref, rtol=2e-5, atol=1e-4):
    y, ref = np.asarray(y, np.float64), np.asarray(ref, np.float64)
    assert y.shape == ref.shape, (y.shape, ref.shape)
    err = np.abs(y - ref) - (rtol * np.abs(ref) + atol)
    assert err.max() <= 0, f"max excess {err.max():.3e}"


def grad_close(g, ref, tol=2e-4, per_row=True, name="", scale=None):
    """Per row (a latent's gradient) or, for parameter gradients — sums over
    the batch with cancellation — relative to the tensor's largest entry
    (`scale`: that entry, when ref holds a sample of the tensor's rows)."""
    g = np.asarray(g, np.float64).reshape(len(ref), -1)
    ref = np.asarray(ref, np.float64).reshape(len(ref), -1)
    if per_row:
        scale = np.abs(ref).max(axis=1, keepdims=True) + 1e-30
    elif scale is None:
        scale = np.abs(ref).max() + 1e-30
    e = (np.abs(g - ref) / scale).max()
    assert e <= tol, f"{name} relative gradient error {e:.3e}"


def word_inputs(z, dev):
    E = synth.word_table(int(z["V"]), 300, seed=int(z["table_seed"]))
    assert float(np.asarray(E, np.float64).sum()) == float(z["table_checksum"])
    wts = torch.tensor(synth.sif_weights(int(z["V"])), dtype=torch.float32, device=dev)
    return torch.tensor(E, device=dev), wts, torch.tensor(z["ids"], device=dev)


def test_word_angular2_golden(gpu, golden):
    import losses

    z = golden("g7_word")
    table, wts, ids = word_inputs(z, gpu)
    x = torch.tensor(z["lat"], device=gpu, requires_grad=True)
    mask = (ids != 0).float()[:, :, None].expand(*ids.shape, 300)
    lp = losses.get_word_log_prob_angular2(x, table, wts[ids], table[ids], mask, 1e-3)
    (lp * torch.tensor(z["up"], device=gpu)).sum().backward()
    close(lp.detach().cpu(), z["lp"])
    grad_close(x.grad.cpu(), z["dlat"])


def test_word_angular_ids_golden(gpu, golden):
    import losses

    z = golden("g7_word_ids")
    table, wts, ids = word_inputs(z, gpu)
    x = torch.tensor(z["lat"], device=gpu, requires_grad=True)
    lp = losses.get_word_log_prob_angular(x, wts, table, ids, (ids != 0).float(), 1e-3)
    (lp * torch.tensor(z["up"], device=gpu)).sum().backward()
    close(lp.detach().cpu(), z["lp"])
    grad_close(x.grad.cpu(), z["dlat"])


@pytest.mark.parametrize("B,V,L", [(37, 3016, 20), (64, 7763, 9), (1, 33, 4), (130, 517, 1)])
def test_word_vs_oracle_shapes(gpu, B, V, L):
    """Ragged tiles: B and V not multiples of 16, one token, one utterance."""
    import latent as LT

    rng = np.random.default_rng(B + V)
    E = synth.word_table(V, 300, seed=V)
    ids = rng.integers(0, V, size=(B, L))
    lat = (0.5 * rng.standard_normal((B, 300))).astype(np.float32)
    w = rng.random((B, L)).astype(np.float32)
    m = (ids != 0).astype(np.float32)
    up = rng.standard_normal(B).astype(np.float32)
    tab = torch.tensor(E)
    xr = torch.tensor(lat, requires_grad=True)
    ref = LO.word_log_prob_angular2(xr, tab, torch.tensor(w), tab[torch.tensor(ids)],
                                    torch.tensor(m)[:, :, None].expand(B, L, 300), 1e-3)
    (ref * torch.tensor(up)).sum().backward()
    wt = LT.word_table(torch.tensor(E, device=gpu))
    x = torch.tensor(lat, device=gpu, requires_grad=True)
    lp = LT.word_log_prob(x, wt, torch.tensor(w, device=gpu), torch.tensor(m, device=gpu), 1e-3,
                          ids=torch.tensor(ids, device=gpu))
    (lp * torch.tensor(up, device=gpu)).sum().backward()
    close(lp.detach().cpu(), ref.detach())
    grad_close(x.grad.cpu(), xr.grad)


@pytest.mark.parametrize("case", ["g7_gauss", "g7_gauss_b1"])
def test_normal_golden(gpu, golden, case):
    import losses

    z = golden(case)
    mu = torch.tensor(z["mu"], device=gpu, requires_grad=True)
    sg = torch.tensor(z["sigma"], device=gpu, requires_grad=True)
    lp = losses.get_normal_log_prob(mu[:, None], sg[:, None], torch.tensor(z["x"], device=gpu),
                                    torch.tensor(z["mask"], device=gpu))
    up = torch.tensor(z["up"], device=gpu)
    (lp * (up[:1] if lp.dim() == 0 else up)).sum().backward()
    close(lp.detach().cpu().numpy(), z["lp"])
    grad_close(mu.grad.cpu(), z["dmu"], 1e-5)
    grad_close(sg.grad.cpu(), z["dsigma"], 1e-5)


def test_log_prob_matrix_golden(gpu, golden):
    import losses
    import models

    z = golden("g8_matrix")
    table, wts, ids = word_inputs(z, gpu)
    B, T = ids.shape
    torch.manual_seed(int(z["gen_seed"]))
    gen = models.AudioVisualGeneratorMultimodal(300, int(z["A"]), int(z["Vd"]), norm="layer_norm",
                                                frozen_weights=False)
    cs = float(np.concatenate([p.detach().numpy().ravel() for p in gen.parameters()])
               .astype(np.float64).sum())
    assert cs == float(z["param_checksum"])  # same construction order -> same seeded weights
    gen = gen.to(gpu)
    text = table[ids]
    tm = (ids != 0).float()[:, :, None].expand(B, T, 300)
    a_, v_ = torch.tensor(z["audio"], device=gpu), torch.tensor(z["visual"], device=gpu)
    am, vm = torch.tensor(z["amask"], device=gpu), torch.tensor(z["vmask"], device=gpu)
    cat = lambda *t: torch.cat(t, -1)
    data = {"text": text, "audio": a_, "visual": v_, "text_weights": wts[ids],
            "audiovisual": cat(a_, v_), "textaudio": cat(text, a_), "textvisual": cat(text, v_),
            "textaudiovisual": cat(text, a_, v_)}
    masks = {"text": tm, "audio": am, "visual": vm, "audiovisual": cat(am, vm),
             "textaudio": cat(tm, am), "textvisual": cat(tm, vm), "textaudiovisual": cat(tm, am, vm)}

    def wfn(latents, word_weights, sent, mask):
        return losses.get_word_log_prob_angular2(latents, table, word_weights, sent, mask, 1e-3)

    x = torch.tensor(z["lat"], device=gpu, requires_grad=True)
    total = losses.get_log_prob_matrix({"word_loss_weight": 0.002}, x, gen(x), data, masks, wfn)
    (-total).mean().backward()
    close(total.detach().cpu(), z["total"])
    grad_close(x.grad.cpu(), z["dlat"])
    for n, p in gen.named_parameters():
        key = "grad_" + n.replace(".", "_")
        g = p.grad.cpu()
        if key + "__rows" in z.files:  # a sample of the rows (tests/golden/slim_goldens.py)
            grad_close(g[z[key + "__rows"]], z[key], per_row=False, name=n,
                       scale=float(z[key + "__absmax"]))
        else:
            grad_close(g, z[key], per_row=False, name=n)


# ------------------------------------------------------------------ CLI
VARIANTS = {
    "e2e_sgd_ln": [],
    "e2e_adam_bn": [],
    "opt_sgd_ln": ["--e2e", "n"],
    "mmb1_e2e": ["--unimodal"],
    "pom_e2e": [],
}


def row_rel(y, ref):
    y, ref = np.asarray(y, np.float64), np.asarray(ref, np.float64)
    return float((np.abs(y - ref).max(1) / np.abs(ref).max(1)).max())


def loss_values(text):
    vals = []
    for line in text.split("\n"):
        line = line.strip().strip("[]")
        vals += [float(v) for v in line.split(",") if v.strip()]
    return np.array(vals)


@pytest.mark.parametrize("graphs", [True, False], ids=["graph_steps", "eager_steps"])
@pytest.mark.parametrize("variant", list(VARIANTS))
def test_cli_matches_reference_run(gpu, tmp_path, monkeypatch, variant, graphs):
    """simplesif.main() against the reference CLI's own run; the optimisation
    steps captured as HIP graphs (the default, simplesif.StepGraphs) and
    launched eagerly."""
    import simplesif

    monkeypatch.setattr(simplesif, "USE_GRAPHS", graphs)
    ref = json.load(open(os.path.join(GOLDEN, f"g9_cli_{variant}.json")))
    arr = np.load(os.path.join(GOLDEN, f"g9_cli_{variant}.npz"))
    dd = ref["data"]
    word2ix, E, splits = synth.mm_splits(dataset=dd["dataset"], n_labels=dd["n_labels"],
                                         seed=dd["seed"], sizes=tuple(dd["sizes"]), T=dd["T"],
                                         V=dd["V"], A_raw=dd["A_raw"], Vd_raw=dd["Vd_raw"])
    wts = synth.sif_weights(E.shape[0])
    monkeypatch.setattr(simplesif, "load_data", lambda args: (word2ix, E.copy(), copy.deepcopy(splits)))
    monkeypatch.setattr(simplesif, "load_weights", lambda args: wts.copy())
    monkeypatch.chdir(tmp_path)
    os.makedirs("configs/golden")
    cfg = ref["config"]
    base = {k: cfg[k] for k in ("sentiment_hidden_size", "lr", "sentiment_lr", "seq_len",
                                "word_sim_metric", "n_epochs", "freeze_weights",
                                "n_sentiment_epochs", "word_loss_weight", "likelihood_weight",
                                "pos_embed_dim", "e2e", "norm", "optimizer", "config_num")}
    (tmp_path / "configs/golden/config_0.json").write_text(json.dumps(base))
    torch.manual_seed(dd["torch_seed"])
    simplesif.main(["configs/golden/config_0.json", dd["dataset"]] + ref["flags"])
    run = tmp_path / "model_saves/golden/config_0_run_0"
    files = sorted(os.path.relpath(os.path.join(dp, f), run) for dp, _, fs in os.walk(run) for f in fs)
    assert files == ref["files"]
    pre = torch.load(run / "pre/embed.bin", weights_only=True).detach().cpu().numpy()
    post = torch.load(run / "post/embed.bin", weights_only=True).detach().cpu().numpy()
    if "rows" in arr.files:  # the fixture keeps every 8th row (tests/golden/slim_goldens.py)
        pre, post = pre[arr["rows"]], post[arr["rows"]]
    e_pre, e_post = row_rel(pre, arr["pre"]), row_rel(post, arr["post"])
    print(f"{variant}: pre {e_pre:.2e} post {e_post:.2e}")
    assert e_pre <= 1e-5
    assert e_post <= 1e-3
    for name, key in (("embed_loss.txt", "embed_loss"), ("embed_valid_loss.txt", "embed_valid_loss"),
                      ("embed_test_loss.txt", "embed_test_loss")):
        got = (run / name).read_text()
        # the non-e2e path writes list reprs (its 'validation losses' are the
        # inner runs' empty validation lists, simplesif.py:148-151)
        assert got.count("[") == ref[key].count("[") and got.count("\n") == ref[key].count("\n")
        if loss_values(ref[key]).size:
            close(loss_values(got), loss_values(ref[key]), rtol=1e-4, atol=1e-3)
        else:
            assert got == ref[key]
    after = json.load(open(run / "post/test_results_after.json"))
    close(np.asarray(after["mae"]), np.asarray(ref["results_after"]["mae"]), rtol=1e-3, atol=1e-4)
    got_cfg = json.load(open(run / "config.json"))
    assert got_cfg == cfg


def test_cli_time_test(gpu, tmp_path, monkeypatch, capsys):
    """--time_test (simplesif.py:808-889): the e2e run, then the closed-form
    MMB2 embeddings of the test split timed, then exit."""
    import simplesif

    ref = json.load(open(os.path.join(GOLDEN, "g9_cli_e2e_sgd_ln.json")))
    dd = ref["data"]
    word2ix, E, splits = synth.mm_splits(seed=dd["seed"], sizes=tuple(dd["sizes"]), T=dd["T"],
                                         V=dd["V"], A_raw=dd["A_raw"], Vd_raw=dd["Vd_raw"])
    monkeypatch.setattr(simplesif, "load_data", lambda args: (word2ix, E.copy(), copy.deepcopy(splits)))
    monkeypatch.setattr(simplesif, "load_weights", lambda args: synth.sif_weights(E.shape[0]))
    monkeypatch.chdir(tmp_path)
    os.makedirs("configs/t")
    cfg = dict(ref["config"])
    (tmp_path / "configs/t/config_0.json").write_text(json.dumps(
        {k: cfg[k] for k in ("sentiment_hidden_size", "lr", "sentiment_lr", "seq_len",
                             "word_sim_metric", "n_epochs", "freeze_weights", "n_sentiment_epochs",
                             "word_loss_weight", "likelihood_weight", "pos_embed_dim", "e2e", "norm",
                             "optimizer", "config_num")}))
    with pytest.raises(SystemExit):
        simplesif.main(["configs/t/config_0.json", "mosi", "--time_test"])
    assert "time taken:" in capsys.readouterr().out
    assert os.path.exists("model_saves/t/config_0_run_0/pre/embed.bin")


def test_fused_generator_and_strided_gaussians(gpu):
    """The generator's twelve linears as one GEMM (per-key mu / sigma column
    views) against the per-key nn.Linear calls of the reference's layout, and
    the strided Gaussian kernels (views passed with their row strides, the
    gradients written into one buffer in the forward's layout) against the
    same kernels on contiguous copies: lp and every gradient equal."""
    import latent as LT
    import models

    torch.manual_seed(5)
    B, A, Vd, T, N = 48, 77, 48, 20, 200
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm="layer_norm",
                                                frozen_weights=False).to(gpu)
    lat = torch.randn(B, 300, device=gpu)
    out = gen(lat)
    x = gen.norm(lat)
    for k, m in gen.embed2out.items():
        close(out[k]["mu"].detach().cpu().numpy(), m["mu"](x).detach().cpu().numpy(), 1e-5, 1e-5)
        close(out[k]["sigma"].detach().cpu().numpy(), m["log_sigma"](x).exp().detach().cpu().numpy(),
              1e-5, 1e-5)
        assert out[k]["mu"].stride(1) == 1 and not out[k]["mu"].is_contiguous()
    g = torch.Generator().manual_seed(3)
    stats = LT.GaussStats(
        text=LT.gauss_stats(torch.randn(N, T, 300, generator=g).to(gpu)),
        audio=LT.gauss_stats(torch.randn(N, T, A, generator=g).to(gpu)),
        visual=LT.gauss_stats(torch.randn(N, T, Vd, generator=g).to(gpu)))
    keys = list(out)
    idx = torch.randint(0, N, (B,), generator=g).to(gpu)
    up = torch.randn(len(keys), B, device=gpu)

    # contiguous copies (the unstrided layout)
    mus_c = [out[k]["mu"].detach().clone().requires_grad_(True) for k in keys]
    sgs_c = [out[k]["sigma"].detach().clone().requires_grad_(True) for k in keys]
    lp_c = LT.gauss_log_prob(stats, keys, mus_c, sgs_c, idx=idx)
    (lp_c * up).sum().backward()
    g_c = [t.grad for t in mus_c + sgs_c]
    # the same values as column blocks of one [B, 2F] (mu) and one [B, F]
    # (sigma) buffer, like the generator's output
    widths = [out[k]["mu"].shape[1] for k in keys]
    f = sum(widths)
    y = torch.zeros(B, 2 * f, device=gpu)
    y[:, :f] = torch.cat([t.detach() for t in mus_c], 1)
    sg_blk = torch.cat([t.detach() for t in sgs_c], 1)
    mus = [t.detach().requires_grad_(True) for t in y[:, :f].split(widths, 1)]
    sgs = [t.detach().requires_grad_(True) for t in sg_blk.split(widths, 1)]
    assert mus[1].stride(0) == 2 * f and sgs[1].stride(0) == f
    lp_s = LT.gauss_log_prob(stats, keys, mus, sgs, idx=idx)
    (lp_s * up).sum().backward()
    assert torch.equal(lp_s.detach(), lp_c.detach())
    for a, b in zip([t.grad for t in mus + sgs], g_c):
        assert torch.equal(a, b)


@pytest.mark.parametrize("n,d", [(0, 300), (1, 300), (64, 300), (1000, 300), (37, 17), (130, 1000)])
def test_layer_norm_backward_matches_torch(n, d):
    """models.LayerNorm (backward: mmb_layer_norm_backward) against torch's
    nn.LayerNorm, both f32 on the device, same parameters and upstream
    gradient: dx per row and dgamma / dbeta within 1e-5 of the tensor's
    largest entry (different reduction order), the forward bit-identical
    (it is torch's)."""
    import models
    gpu = torch.device("cuda:0")
    g = torch.Generator().manual_seed(n * 7 + d)
    x = (torch.randn(n, d, generator=g) * 3 + 1).to(gpu)
    dy = torch.randn(n, d, generator=g).to(gpu)
    ours, ref = models.LayerNorm(d).to(gpu), torch.nn.LayerNorm(d).to(gpu)
    with torch.no_grad():
        w, b = torch.randn(d, generator=g), torch.randn(d, generator=g)
        for m in (ours, ref):
            m.weight.copy_(w)
            m.bias.copy_(b)
    outs = []
    for m in (ours, ref):
        xi = x.clone().requires_grad_(True)
        y = m(xi)
        y.backward(dy)
        outs.append((y.detach(), xi.grad, m.weight.grad, m.bias.grad))
    (y, dx, dw, db), (y_r, dx_r, dw_r, db_r) = outs
    assert torch.equal(y, y_r)
    if n:
        err = (dx - dx_r).abs().amax(1) / dx_r.abs().amax(1).clamp_min(1e-30)
        assert err.max().item() <= 1e-5
    for a, r in ((dw, dw_r), (db, db_r)):
        assert (a - r).abs().max().item() <= 1e-5 * max(r.abs().max().item(), 1e-30)
