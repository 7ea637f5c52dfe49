"""Golden fixtures for the latent-optimisation row and
the simplesif.py CLI, made by running the REFERENCE in the build container:

    python tests/golden/make_goldens_latent.py

Imports the reference's `losses`, `models` and `simplesif` (behind an h5py
stub and an `analyze_embeddings` stub whose get_closest_words returns []; both
are used only for file loading / printing) and records inputs/outputs as small
.npz/.json files.  Only data is committed — no reference source.  Word tables
and datasets are regenerated from seeds by `multimodal-baselines_amd/synth.py`
(checksums stored).

  g7_word          get_word_log_prob_angular2 (losses.py:68-95): lp and d lp/d latents
  g7_word_ids      get_word_log_prob_angular (losses.py:36-66) on id input
  g7_gauss         get_normal_log_prob (losses.py:13-33): lp, d/d mu, d/d sigma
  g7_gauss_b1      the same at B = 1 (the .squeeze() quirk: a scalar)
  g8_matrix        get_log_prob_matrix (losses.py:216-274) over a seeded
                   AudioVisualGeneratorMultimodal (layer_norm): total, grads
  g10_utils        utils.normalize_data / add_positional_embeddings on a seeded split
  g9_cli_<variant> simplesif.main() end to end on seeded mm_splits data
                   (load_data / load_weights replaced by the seeded splits):
                   pre/post embed.bin, loss files, regressor results
"""
from __future__ import annotations

import importlib.util
import json
import os
import shutil
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


synth = _load("amd_synth", os.path.join(REPO, "multimodal-baselines_amd", "synth.py"))

sys.path.insert(0, REF)
sys.modules.setdefault("h5py", types.ModuleType("h5py"))
_ae = types.ModuleType("analyze_embeddings")
_ae.get_closest_words = lambda *a, **k: []
sys.modules.setdefault("analyze_embeddings", _ae)
import torch  # noqa: E402
import losses as R_losses  # noqa: E402
import models as R_models  # noqa: E402

CLI_DATA = dict(seed=5, sizes=(96, 32, 32), T=12, V=300, A_raw=20, Vd_raw=14)


def checksum(a) -> float:
    return float(np.asarray(a, dtype=np.float64).sum())


def save(name, **arrs):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrs)
    print("wrote", path, sorted(arrs))


def word_case():
    V, B, Lt = 517, 48, 20
    E = synth.word_table(V, 300, seed=71)
    wts = synth.sif_weights(V)
    rng = np.random.default_rng(72)
    ids = rng.integers(1, V, size=(B, Lt)).astype(np.int64)
    lens = rng.integers(3, Lt + 1, size=B)
    ids[np.arange(Lt)[None, :] >= lens[:, None]] = 0
    lat = (0.5 * rng.standard_normal((B, 300)) + 0.3 * E[ids[:, 0]]).astype(np.float32)
    up = rng.standard_normal(B).astype(np.float32)
    table = torch.tensor(E)
    wt = torch.tensor(wts, dtype=torch.float32)
    idt = torch.tensor(ids)
    # angular2 (the CLI's word model): dense sentence rows + [B, L, 300] mask
    x = torch.tensor(lat, requires_grad=True)
    mask = (idt != 0).to(torch.int64).unsqueeze(-1).expand(B, Lt, 300).float()
    lp = R_losses.get_word_log_prob_angular2(x, table, wt[idt], table[idt], mask, 1e-3)
    (lp * torch.tensor(up)).sum().backward()
    save("g7_word", ids=ids, lat=lat, up=up, lp=lp.detach().numpy(), dlat=x.grad.numpy(),
         V=V, table_seed=71, table_checksum=checksum(E))
    # angular (ids + [B, L] mask)
    x = torch.tensor(lat, requires_grad=True)
    m2 = (idt != 0).float()
    lp = R_losses.get_word_log_prob_angular(x, wt, table, idt, m2, 1e-3)
    (lp * torch.tensor(up)).sum().backward()
    save("g7_word_ids", ids=ids, lat=lat, up=up, lp=lp.detach().numpy(), dlat=x.grad.numpy(),
         V=V, table_seed=71, table_checksum=checksum(E))


def gauss_case(name, B, T, F, seed):
    rng = np.random.default_rng(seed)
    mu = rng.standard_normal((B, F)).astype(np.float32)
    sg = np.exp(0.3 * rng.standard_normal((B, F))).astype(np.float32)
    x = rng.standard_normal((B, T, F)).astype(np.float32)
    m = (rng.random((B, T, F)) > 0.2).astype(np.float32)
    up = rng.standard_normal(B).astype(np.float32)
    tm = torch.tensor(mu, requires_grad=True)
    ts = torch.tensor(sg, requires_grad=True)
    lp = R_losses.get_normal_log_prob(tm.unsqueeze(1), ts.unsqueeze(1), torch.tensor(x), torch.tensor(m))
    (lp * torch.tensor(up[:1] if lp.dim() == 0 else up)).sum().backward()
    save(name, mu=mu, sigma=sg, x=x, mask=m, up=up, lp=lp.detach().numpy(),
         dmu=tm.grad.numpy(), dsigma=ts.grad.numpy())


def matrix_case():
    V, B, T, A, Vd = 517, 24, 10, 28, 20
    E = synth.word_table(V, 300, seed=81)
    wts = synth.sif_weights(V)
    rng = np.random.default_rng(82)
    ids = rng.integers(1, V, size=(B, T)).astype(np.int64)
    ids[:, :2] = 0
    aud = rng.standard_normal((B, T, A)).astype(np.float32)
    vis = rng.standard_normal((B, T, Vd)).astype(np.float32)
    am = (rng.random((B, T, A)) > 0.1).astype(np.float32)
    vm = (rng.random((B, T, Vd)) > 0.1).astype(np.float32)
    lat = (0.5 * rng.standard_normal((B, 300))).astype(np.float32)
    torch.manual_seed(83)
    gen = R_models.AudioVisualGeneratorMultimodal(300, A, Vd, norm="layer_norm", frozen_weights=False)
    table = torch.tensor(E)
    wt = torch.tensor(wts, dtype=torch.float32)
    idt = torch.tensor(ids)
    text = table[idt]
    tm = (idt != 0).to(torch.int64).unsqueeze(-1).expand(B, T, 300).float()
    a_, v_ = torch.tensor(aud), torch.tensor(vis)
    am_, vm_ = torch.tensor(am), torch.tensor(vm)
    data = {"text": text, "audio": a_, "visual": v_, "text_weights": wt[idt],
            "audiovisual": torch.cat([a_, v_], -1), "textaudio": torch.cat([text, a_], -1),
            "textvisual": torch.cat([text, v_], -1), "textaudiovisual": torch.cat([text, a_, v_], -1)}
    masks = {"text": tm, "audio": am_, "visual": vm_, "audiovisual": torch.cat([am_, vm_], -1),
             "textaudio": torch.cat([tm, am_], -1), "textvisual": torch.cat([tm, vm_], -1),
             "textaudiovisual": torch.cat([tm, am_, vm_], -1)}

    def wfn(latents, word_weights, sent, mask):  # simplesif.py:527-537
        return R_losses.get_word_log_prob_angular2(latents, table, word_weights, sent, mask, 1e-3)

    x = torch.tensor(lat, requires_grad=True)
    out = gen(x)
    total = R_losses.get_log_prob_matrix({"word_loss_weight": 0.002}, x, out, data, masks, wfn)
    (-total).mean().backward()
    grads = {f"grad_{n.replace('.', '_')}": p.grad.numpy() for n, p in gen.named_parameters()}
    params = {"param_checksum": checksum(np.concatenate([p.detach().numpy().ravel()
                                                         for p in gen.parameters()]))}
    save("g8_matrix", ids=ids, audio=aud, visual=vis, amask=am, vmask=vm, lat=lat,
         total=total.detach().numpy(), dlat=x.grad.numpy(), V=V, A=A, Vd=Vd, table_seed=81,
         table_checksum=checksum(E), gen_seed=83, **grads, **params)


def cli_case(variant, cfg, flags, dataset="mosi", n_labels=1, seed=1234):
    import simplesif as R_ss

    word2ix, E, splits = synth.mm_splits(dataset=dataset, n_labels=n_labels, **CLI_DATA)
    wts = synth.sif_weights(E.shape[0])

    def load_data(args):
        import copy
        return word2ix, E.copy(), copy.deepcopy(splits)

    R_ss.load_data = load_data
    R_ss.load_weights = lambda args: wts.copy()
    work = tempfile.mkdtemp(prefix="mmb_cli_")
    cwd = os.getcwd()
    try:
        os.chdir(work)
        os.makedirs("configs/golden", exist_ok=True)
        with open("configs/golden/config_0.json", "w") as f:
            json.dump(cfg, f)
        sys.argv = ["simplesif.py", "configs/golden/config_0.json", dataset] + flags
        torch.manual_seed(seed)
        R_ss.main()
        run = os.path.join("model_saves", "golden", "config_0_run_0")
        ld = lambda p: torch.load(os.path.join(run, p), weights_only=True).detach().numpy()
        rd = lambda p: open(os.path.join(run, p)).read()  # raw text (some hold list reprs)
        arrs = {"pre": ld("pre/embed.bin"), "post": ld("post/embed.bin")}
        js = {"embed_loss": rd("embed_loss.txt"), "embed_valid_loss": rd("embed_valid_loss.txt"),
              "embed_test_loss": rd("embed_test_loss.txt"),
              "senti_train_loss": rd("post/senti_train_loss.txt"),
              "senti_valid_loss": rd("post/senti_valid_loss.txt"),
              "results_before": json.load(open(os.path.join(run, "post/test_results_before.json"))),
              "results_after": json.load(open(os.path.join(run, "post/test_results_after.json"))),
              "config": json.load(open(os.path.join(run, "config.json"))),
              "files": sorted(os.path.relpath(os.path.join(dp, f), run)
                              for dp, _, fs in os.walk(run) for f in fs),
              "data": dict(CLI_DATA, dataset=dataset, n_labels=n_labels, torch_seed=seed),
              "flags": flags}
    finally:
        os.chdir(cwd)
        shutil.rmtree(work, ignore_errors=True)
    save("g9_cli_" + variant, **arrs)
    with open(os.path.join(HERE, "g9_cli_" + variant + ".json"), "w") as f:
        json.dump(js, f, indent=1, sort_keys=True)


BASE_CFG = {"sentiment_hidden_size": 100, "lr": 1e-3, "sentiment_lr": 0.1, "seq_len": 20,
            "word_sim_metric": "angular", "n_epochs": 2, "freeze_weights": False,
            "n_sentiment_epochs": 3, "word_loss_weight": 0.001, "likelihood_weight": 0.001,
            "pos_embed_dim": 2, "e2e": True, "norm": "layer_norm", "optimizer": "sgd",
            "config_num": 0}


def utils_case():
    import copy

    import utils as R_utils

    _, _, (tr, va, te) = synth.mm_splits(seed=11, sizes=(40, 8, 8), T=9, V=50, A_raw=7, Vd_raw=5)
    d, m = R_utils.normalize_data(copy.deepcopy(tr))
    pe2 = R_utils.add_positional_embeddings({"pos_embed_dim": 2}, d["covarep"])
    pe4 = R_utils.add_positional_embeddings({"pos_embed_dim": 4}, d["facet"])
    save("g10_utils", covarep=d["covarep"], facet=d["facet"], cov_mask=m["covarep"],
         fac_mask=m["facet"], pe2=pe2, pe4=pe4)


def main():
    torch.set_num_threads(8)
    utils_case()
    word_case()
    gauss_case("g7_gauss", 16, 12, 37, 91)
    gauss_case("g7_gauss_b1", 1, 12, 37, 92)
    matrix_case()
    cli_case("e2e_sgd_ln", dict(BASE_CFG), [])
    cli_case("e2e_adam_bn", dict(BASE_CFG, optimizer="adam", norm="batch_norm", lr=1e-4), [])
    # the non-e2e objective is the raw -log p (T x F frames, no likelihood weight):
    # at the grid's lr = 1e-3 plain SGD diverges to NaN on this data, so 1e-6
    cli_case("opt_sgd_ln", dict(BASE_CFG, lr=1e-6), ["--e2e", "n"])
    cli_case("mmb1_e2e", dict(BASE_CFG, pos_embed_dim=4), ["--unimodal"])
    cli_case("pom_e2e", dict(BASE_CFG), [], dataset="pom", n_labels=3)


if __name__ == "__main__":
    main()
