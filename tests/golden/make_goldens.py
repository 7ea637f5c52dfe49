"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

Run in the build container only (needs /root/reference, read-only):

    python tests/golden/make_goldens.py

It imports the reference's own hot-path functions (`sif_functions`, `sif`,
`sif2` behind an h5py stub, `sentiment_model`, `losses`) and records their
inputs and outputs as small .npz/.json files.  Only data is committed — no
reference source.  Large inputs (word tables, frame streams, generator
weights) are NOT stored; they are regenerated from the seeds recorded in each
fixture by `multimodal-baselines_amd/synth.py` / `models.py`, and each fixture
carries a float64 checksum of every regenerated input so drift is detected.

Fixtures:
  g1_pom_valid / g1_pom_test  a1-a5 on real POM ids + real POM weights,
                              synthetic V=7763 table, N<300 (transposed
                              randomized-SVD branch)
  g2_mosi                     a1-a5 MOSI-like, N=512 >= 300 (direct branch)
  g3_gap                      a3 stress: iid table, s1/s2 ~ 1.07
  g3b_npc2                    remove_pc with npc=2
  g1c_seq2weight              a1 with a random mask and negative ids
  g4_mmb2_mosi / g4_mmb2_syn  a7/a8 closed-form MMB2 (f32 and f64 runs)
  g5_senti                    a10/a11: one SGD step + a 20-epoch train run
  g6_metrics                  a12 metric dicts
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
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
amd_models = _load("amd_models", os.path.join(REPO, "multimodal-baselines_amd", "models.py"))

sys.path.insert(0, REF)
sys.modules.setdefault("h5py", types.ModuleType("h5py"))  # only used for file loading (utils.py:35)
import torch  # noqa: E402
import sif_functions as R_sf  # noqa: E402
import sif as R_sif  # noqa: E402
import sif2 as R_sif2  # noqa: E402
import sentiment_model as R_sm  # noqa: E402
import losses as R_losses  # noqa: E402
import models as R_models  # noqa: E402


def checksum(a) -> float:
    return float(np.asarray(a, dtype=np.float64).sum())


def f32_exact(x):
    """a2's f64 output holds f32 values (sif_functions.py:55): store it losslessly as f32."""
    y = np.asarray(x).astype(np.float32)
    assert np.array_equal(y.astype(np.float64), x)
    return y


def spectral_ratio(X):
    s = np.linalg.svd(np.asarray(X, np.float64), compute_uv=False)
    return float(s[0] / s[1])


def save(name, **arrs):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrs)
    print(f"wrote {path} ({os.path.getsize(path)} B)")


def sif_case(name, ids, weights, table_seed, V, D=300, common=0.3, note=""):
    E = synth.word_table(V, D, seed=table_seed, common=common)
    w = R_sif.get_sentence_word_weights(ids, weights)                 # a1
    emb = R_sf.get_weighted_average(E, ids, w)                        # a2
    pc = R_sf.compute_pc(emb, 1)                                      # a3
    out = R_sif.get_sentence_embeddings(E, weights, ids)              # a1-a5
    save(name, ids=ids, weights=weights, table_seed=np.int64(table_seed), V=np.int64(V),
         D=np.int64(D), common=np.float64(common), table_checksum=np.float64(checksum(E)),
         w=w, emb=f32_exact(emb), pc=pc, out=out, s1_s2=np.float64(spectral_ratio(emb)), note=note)


def main():
    # ---- G1: real POM ids + weights (sif.py:34-46 loads pom/pom_word_weights.npy)
    pom_w = np.load(os.path.join(REF, "pom", "pom_word_weights.npy")).squeeze()
    valid = np.load(os.path.join(REF, "pom", "pom_valid_ids.npy"))
    test = np.load(os.path.join(REF, "pom", "pom_test_ids.npy"))
    sif_case("g1_pom_valid", valid[:64], pom_w, table_seed=1, V=7763,
             note="pom_valid_ids rows 0-63, real POM weights")
    sif_case("g1_pom_test", test[:48], pom_w, table_seed=2, V=7763,
             note="pom_test_ids rows 0-47, real POM weights")

    # ---- G2: MOSI-like, N >= 300 (randomized_svd direct branch)
    V2 = 3016
    ids2 = synth.token_ids(320, 20, V2, seed=3, ragged=True)
    w2 = synth.sif_weights(V2, w0=0.0)
    sif_case("g2_mosi", ids2, w2, table_seed=4, V=V2, note="MOSI shape, ragged, w[0]=0")

    # ---- G3: no spectral gap (iid table) — randomized SVD != exact SVD here
    ids3 = synth.token_ids(320, 16, 2000, seed=5)
    w3 = synth.sif_weights(2000, w0=1.0)
    sif_case("g3_gap", ids3, w3, table_seed=6, V=2000, common=0.0, note="iid table, s1/s2~1")

    # ---- G3b: npc = 2 (remove_pc generic branch, sif_functions.py:79-80)
    E = synth.word_table(1500, 300, seed=7)
    ids = synth.token_ids(320, 24, 1500, seed=8, ragged=True)
    wt = synth.sif_weights(1500)
    w = R_sif.get_sentence_word_weights(ids, wt)
    emb = R_sf.get_weighted_average(E, ids, w)
    pc2 = R_sf.compute_pc(emb, 2)
    out2 = R_sf.remove_pc(emb, 2)
    save("g3b_npc2", ids=ids, weights=wt, table_seed=np.int64(7), V=np.int64(1500),
         D=np.int64(300), common=np.float64(0.3), table_checksum=np.float64(checksum(E)),
         emb=f32_exact(emb), pc=pc2, out=out2)

    # ---- G1c: seq2weight with mask and negative ids (sif_functions.py:8-15)
    rng = np.random.default_rng(9)
    seq = rng.integers(-3, 500, size=(40, 33)).astype(np.int64)
    mask = (rng.random((40, 33)) > 0.2).astype(np.float64)
    wt = synth.sif_weights(500)
    wout = R_sf.seq2weight(seq, mask, wt)
    # weighted average with negative ids (numpy wraps We[-1]) and given weights
    E = synth.word_table(500, 300, seed=10)
    emb = R_sf.get_weighted_average(E, seq, wout)
    save("g1c_seq2weight", seq=seq, mask=mask, weights=wt, w=wout, table_seed=np.int64(10),
         V=np.int64(500), D=np.int64(300), common=np.float64(0.3),
         table_checksum=np.float64(checksum(E)), emb=f32_exact(emb))

    # ---- G4: closed-form MMB2 (sif2.py:103-114, 164-208)
    for name, N, T, A, Vd, V, pe in (("g4_mmb2_mosi", 64, 20, 76, 48, 3016, 0.3),
                                      ("g4_mmb2_syn", 16, 40, 300, 300, 4000, 0.0)):
        torch.manual_seed(0)
        gen = R_models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None, frozen_weights=True)
        torch.manual_seed(0)
        ours = amd_models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None, frozen_weights=True)
        for (k1, p1), (k2, p2) in zip(gen.state_dict().items(), ours.state_dict().items()):
            assert k1 == k2 and torch.equal(p1, p2), (k1, k2)
        E = synth.word_table(V, 300, seed=11)
        ids = synth.token_ids(N, T, V, seed=12, ragged=True, min_len=T // 2)
        wt = synth.sif_weights(V)
        audio = synth.frames(N, T, A, seed=13, pad_frac=pe)
        visual = synth.frames(N, T, Vd, seed=14, pad_frac=pe)
        outs = {}
        for dt in (torch.float32, torch.float64):
            Et = torch.tensor(E, dtype=dt)
            wtt = torch.tensor(wt, dtype=torch.float32).to(dt)  # simplesif.py:315 f32 rounding
            idt = torch.as_tensor(ids, dtype=torch.long)
            text = Et[idt]
            au = torch.tensor(audio, dtype=dt)
            vi = torch.tensor(visual, dtype=dt)
            data = {"text": text, "audio": au, "visual": vi,
                    "audiovisual": torch.cat([au, vi], -1),
                    "textaudio": torch.cat([text, au], -1),
                    "textvisual": torch.cat([text, vi], -1),
                    "textaudiovisual": torch.cat([text, au, vi], -1)}
            masks = {k: None for k in data}
            g = gen.to(dt)
            nets = {k: (g.embed2out[k]["mu"], g.embed2out[k]["log_sigma"]) for k in amd_models.MMB2_KEYS}
            sw = torch.zeros(ids.shape, dtype=dt)
            for i in range(N):                                     # simplesif.py:867-868
                sw[i] = torch.gather(wtt, 0, idt[i])
            with torch.no_grad():
                cs = R_sif2.estimate_embedding_overall_gpu2(data, masks, nets, sw, text)
            outs[str(dt).split(".")[-1]] = cs.numpy()
            if dt == torch.float32:
                qm, qs = R_sif2.calc_weights(au, nets["audio"][0].bias, nets["audio"][1].bias, None)
                calc_qm, calc_qs = qm[:4].numpy(), qs[:4].numpy()
        save(name, ids=ids, weights=wt, V=np.int64(V), A=np.int64(A), Vd=np.int64(Vd),
             table_seed=np.int64(11), table_checksum=np.float64(checksum(E)),
             audio_seed=np.int64(13), visual_seed=np.int64(14), pad_frac=np.float64(pe),
             audio_checksum=np.float64(checksum(audio)), visual_checksum=np.float64(checksum(visual)),
             param_checksums=np.array([checksum(p.detach().numpy()) for p in gen.float().state_dict().values()]),
             cs_f32=outs["float32"], cs_f64=outs["float64"], calc_qm_audio=calc_qm,
             calc_qs_audio=calc_qs)

    # ---- G5: regressor (sentiment_model.py:29-41, 76-163)
    torch.manual_seed(0)
    model = R_sm.SentimentModel(300, 100, 1)
    x = torch.tensor(np.random.default_rng(15).standard_normal((32, 300)).astype(np.float32))
    y = torch.tensor(np.random.default_rng(16).uniform(-3, 3, 32).astype(np.float32))
    w1, b1 = model.hidden1.weight.detach().clone(), model.hidden1.bias.detach().clone()
    w2, b2 = model.out.weight.detach().clone(), model.out.bias.detach().clone()
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    model.zero_grad()
    pred = model(x)
    loss = torch.nn.L1Loss(reduction="none")(pred, y)
    loss.mean().backward()
    g = [p.grad.detach().clone() for p in (model.hidden1.weight, model.hidden1.bias,
                                             model.out.weight, model.out.bias)]
    opt.step()
    save("g5_senti_step", x=x.numpy(), y=y.numpy(), w1=w1.numpy(), b1=b1.numpy(), w2=w2.numpy(),
         b2=b2.numpy(), pred=pred.detach().numpy(), loss=np.float64(loss.mean().item()),
         gw1=g[0].numpy(), gb1=g[1].numpy(), gw2=g[2].numpy(), gb2=g[3].numpy(),
         nw1=model.hidden1.weight.detach().numpy(), nb1=model.hidden1.bias.detach().numpy(),
         nw2=model.out.weight.detach().numpy(), nb2=model.out.bias.detach().numpy())

    # 20-epoch train_sentiment_for_latents run, MOSI-like split sizes scaled down
    rng = np.random.default_rng(17)
    lat = [rng.standard_normal((n, 300)).astype(np.float32) for n in (200, 50, 70)]
    wproj = rng.standard_normal(300).astype(np.float32) / 8
    labels = [np.clip(l @ wproj + 0.3 * rng.standard_normal(l.shape[0]), -3, 3).astype(np.float32)
              for l in lat]
    args = {"sentiment_hidden_size": 100, "n_sentiment_epochs": 20, "sentiment_lr": 0.1,
            "early_stopping": False, "dataset": "mosi", "lr_decay": 0.5}
    torch.manual_seed(1234)
    captured = {}
    orig = R_sm.train_sentiment

    def spy(*a, **k):
        tl, vl = orig(*a, **k)
        captured["train"] = [float(t) for t in tl]
        captured["valid"] = [float(t) for t in vl]
        captured["model"] = {kk: v.detach().clone() for kk, v in a[1].state_dict().items()}
        return tl, vl

    metrics = []
    orig_fl = R_sm.full_loss

    def spy_fl(p, y):
        r = orig_fl(p, y)
        metrics.append(r)
        return r

    R_sm.train_sentiment = spy
    R_sm.full_loss = spy_fl
    import io
    import contextlib
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        R_sm.train_sentiment_for_latents(args, tuple(torch.tensor(l) for l in lat),
                                          tuple(labels), torch.device("cpu"))
    R_sm.train_sentiment = orig
    R_sm.full_loss = orig_fl
    with open(os.path.join(HERE, "g5_senti_train_metrics.json"), "w") as f:
        json.dump({"before": metrics[0], "after": metrics[1]}, f, indent=1, sort_keys=True)
    # the final metrics are printed by full_loss; recompute them from the model
    save("g5_senti_train", lat_train=lat[0], lat_valid=lat[1], lat_test=lat[2],
         y_train=labels[0], y_valid=labels[1], y_test=labels[2], seed=np.int64(1234),
         train_losses=np.array(captured["train"]), valid_losses=np.array(captured["valid"]),
         **{"final_" + k.replace(".", "_"): v.numpy() for k, v in captured["model"].items()})

    # ---- G6: metrics (losses.py:276-366)
    rng = np.random.default_rng(18)
    pred = rng.uniform(-3, 3, 120).astype(np.float32)
    yt = np.clip(pred + rng.normal(0, 1, 120), -3, 3).astype(np.float32)
    predp = rng.uniform(1, 7, (90, 4)).astype(np.float32)
    ytp = np.clip(predp + rng.normal(0, 1, (90, 4)), 1, 7).astype(np.float32)
    predi = rng.standard_normal((80, 2)).astype(np.float32)
    yti = np.eye(2, dtype=np.float32)[rng.integers(0, 2, 80)]
    with contextlib.redirect_stdout(io.StringIO()):
        res = {"full": R_losses.full_loss(pred, yt), "pom": R_losses.pom_loss(predp, ytp),
               "iemocap": R_losses.iemocap_loss(predi, yti)}
    save("g6_metrics_inputs", pred=pred, y=yt, pred_pom=predp, y_pom=ytp, pred_iemocap=predi,
         y_iemocap=yti)
    with open(os.path.join(HERE, "g6_metrics.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("done")


if __name__ == "__main__":
    main()
