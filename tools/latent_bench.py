#!/usr/bin/env python3
"""Step time of the e2e latent-optimisation loop at MOSI shape.

    python tools/latent_bench.py [--steps 50] [--cpu-steps 3] [--vocab 3016] [--batch 64]

One step = simplesif.py:712-790 for one batch: generator forward (layer_norm +
12 linears), the objective (word model over the whole vocabulary + six
Gaussian combinations), the regressor, backward, SGD on latents + generator
+ regressor.  Three implementations of the objective on the same inputs:

  libmmb   simplesif.Objective (HIP kernels, frame sums precomputed per split)
  eager    the reference's torch arithmetic on the GPU (oracle/latent_oracle,
           the [B, V, 300] broadcast and [B, T, F] Gaussians rebuilt per step)
  cpu      the same reference arithmetic on the host cores (bounded sample)

Prints one JSON line (ms per step, steps/s).
"""
import argparse
import copy
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-baselines_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def build(args, dev):
    import latent as LT
    import models
    import simplesif
    import synth
    import utils
    from sentiment_model import SentimentModel

    w2i, E, (tr, _, _) = synth.mm_splits(seed=1, sizes=(args.n, 8, 8), T=args.t, V=args.vocab,
                                         A_raw=args.a, Vd_raw=args.vd)
    tr, m = utils.normalize_data(tr)
    pe = {"pos_embed_dim": 2}
    tr["covarep"] = utils.add_positional_embeddings(pe, tr["covarep"])
    tr["facet"] = utils.add_positional_embeddings(pe, tr["facet"])
    ext = np.ones(tr["covarep"].shape[:2] + (2,), np.int64)
    m["covarep"] = np.concatenate([m["covarep"], ext], -1)
    m["facet"] = np.concatenate([m["facet"], ext], -1)
    wts = torch.tensor(synth.sif_weights(args.vocab), dtype=torch.float32, device=dev)
    table = torch.tensor(E, device=dev)
    ids = torch.tensor(tr["text"], device=dev)
    gm = (ids != 0).float()[:, :, None]
    cfg = {"word_loss_weight": 0.001, "likelihood_weight": 0.001}
    obj = simplesif.Objective(cfg, LT.word_table(table), wts, tr["text"], table[ids], gm,
                              tr["covarep"], m["covarep"], tr["facet"], m["facet"])
    A, Vd = tr["covarep"].shape[-1], tr["facet"].shape[-1]
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm="layer_norm", frozen_weights=False)
    senti = SentimentModel(300, 100, 1)
    lat0 = torch.randn(args.n, 300) * 0.5
    label = torch.tensor(tr["label"])
    data = dict(ids=ids, table=table, wts=wts, audio=torch.tensor(tr["covarep"], dtype=torch.float32),
                visual=torch.tensor(tr["facet"], dtype=torch.float32),
                amask=torch.tensor(m["covarep"], dtype=torch.float32),
                vmask=torch.tensor(m["facet"], dtype=torch.float32))
    return cfg, obj, gen, senti, lat0, label, data


def eager_objective(cfg, data, dev):
    """The reference's per-batch objective (simplesif.py:93-131 + losses.py) in torch."""
    from oracle import latent_oracle as LO

    table = data["table"].to(dev)
    ids = data["ids"].to(dev)
    wts = data["wts"].to(dev)
    audio, visual = data["audio"].to(dev), data["visual"].to(dev)
    am, vm = data["amask"].to(dev), data["vmask"].to(dev)

    def f(lat, out, j):
        idj = ids[j]
        text = table[idj]
        tm = (idj != 0).float()[:, :, None].expand(*idj.shape, 300)
        a, v, a_m, v_m = audio[j], visual[j], am[j], vm[j]
        cat = lambda *t: torch.cat(t, -1)
        bd = {"text": text, "audio": a, "visual": v, "text_weights": wts[idj],
              "audiovisual": cat(a, v), "textaudio": cat(text, a), "textvisual": cat(text, v),
              "textaudiovisual": cat(text, a, v)}
        bm = {"text": tm, "audio": a_m, "visual": v_m, "audiovisual": cat(a_m, v_m),
              "textaudio": cat(tm, a_m), "textvisual": cat(tm, v_m), "textaudiovisual": cat(tm, a_m, v_m)}
        wfn = lambda l, w, s, m: LO.word_log_prob_angular2(l, table, w, s, m, 1e-3)
        return LO.log_prob_matrix(cfg, lat, out, bd, bm, wfn)
    return f


def run(cfg, objective, gen, senti, lat0, label, dev, steps, batch, warm=2, graph_obj=None):
    """ms per e2e step.  graph_obj (a simplesif.Objective): the step as the
    CLI runs it by default -- device work captured in a HIP graph
    (simplesif.StepGraphs), one host read for the reference's checks, eager
    optimiser step."""
    gen = gen.to(dev)
    senti = senti.to(dev)
    lat = lat0.clone().to(dev).requires_grad_(True)
    lab = label.to(dev)
    params = [lat] + list(gen.parameters()) + list(senti.parameters())
    opt = torch.optim.SGD(params, lr=1e-3)
    l1 = torch.nn.L1Loss(reduction="none")
    g = torch.Generator().manual_seed(0)
    n = lat.shape[0]

    if graph_obj is not None:
        import simplesif

        lw = cfg["likelihood_weight"]

        def body(j):
            e = lat[j]  # one gather (simplesif's graph body)
            out = gen(e)
            sig = simplesif.sigma_mins(out)
            lp, mins = graph_obj.log_prob_nocheck(e, out, j)
            sl = l1(senti(e), lab[j]).mean(dim=-1)
            lm = (lw * (-lp) + (1 - lw) * sl).mean()
            lm.backward()
            return out, torch.cat([lm.detach().view(1), sig, mins])

        graphs = simplesif.StepGraphs(body, [gen, senti], params, dev)

        def gstep():
            j = torch.randperm(n, generator=g)[:batch]
            out, vals = graphs.step(j, opt)
            return simplesif.check_step(out, vals, lat[:batch].size(), len(vals) - 2 - len(out))

        for _ in range(warm):
            gstep()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            gstep()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    def step():
        j = torch.randperm(n, generator=g)[:batch].to(dev)
        opt.zero_grad()
        out = gen(lat[j])
        lp = -objective(lat[j], out, j)
        sl = l1(senti(lat[j]), lab[j]).mean(dim=-1)
        loss = cfg["likelihood_weight"] * lp + (1 - cfg["likelihood_weight"]) * sl
        loss.mean().backward()
        opt.step()
        return loss

    for _ in range(warm):
        step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def plain_torch(gen):
    """A copy of the generator with every models.LayerNorm (libmmb backward on
    the device) swapped for torch's nn.LayerNorm: the reference's arithmetic
    for the torch legs."""
    import models

    g = copy.deepcopy(gen)
    for name, mod in list(g.named_modules()):
        for cname, child in list(mod.named_children()):
            if isinstance(child, models.LayerNorm):
                ln = torch.nn.LayerNorm(child.normalized_shape, eps=child.eps,
                                        elementwise_affine=child.elementwise_affine)
                ln.load_state_dict(child.state_dict())
                setattr(mod, cname, ln.to(next(child.parameters()).device))
    return g


class CpuSenti(torch.nn.Module):  # the reference regressor in plain torch (no libmmb on CPU)
    def __init__(self, m):
        super().__init__()
        self.h = torch.nn.Linear(300, 100)
        self.o = torch.nn.Linear(100, 1)
        with torch.no_grad():
            self.h.weight.copy_(m.hidden1.weight.cpu()), self.h.bias.copy_(m.hidden1.bias.cpu())
            self.o.weight.copy_(m.out.weight.cpu()), self.o.bias.copy_(m.out.bias.cpu())

    def forward(self, x):
        return self.o(torch.relu(self.h(x))).squeeze()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--n", type=int, default=1284)
    ap.add_argument("--t", type=int, default=20)
    ap.add_argument("--vocab", type=int, default=3016)
    ap.add_argument("--a", type=int, default=75)
    ap.add_argument("--vd", type=int, default=46)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--only-graph", action="store_true",
                    help="time the graph step alone (for a kernel trace of just that path)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg, obj, gen, senti, lat0, label, data = build(args, dev)
    import copy

    if args.only_graph:
        ms_graph = run(cfg, None, copy.deepcopy(gen), copy.deepcopy(senti), lat0, label, dev,
                       args.steps, args.batch, graph_obj=obj)
        print(json.dumps({"ms_per_step": {"libmmb_graph": round(ms_graph, 4)}, "steps": args.steps}))
        return

    ms_hip = run(cfg, obj.log_prob, copy.deepcopy(gen), copy.deepcopy(senti), lat0, label, dev,
                 args.steps, args.batch)
    ms_graph = run(cfg, None, copy.deepcopy(gen), copy.deepcopy(senti), lat0, label, dev,
                   args.steps, args.batch, graph_obj=obj)

    ms_eager = run(cfg, eager_objective(cfg, data, dev), plain_torch(gen).float(),
                   CpuSenti(senti), lat0, label, dev, args.steps, args.batch)
    cpu = torch.device("cpu")
    from oracle import latent_oracle as LO  # noqa: F401  (cpu leg: the reference arithmetic)

    ms_cpu = run(cfg, eager_objective(cfg, data, cpu), plain_torch(gen).cpu(), CpuSenti(senti),
                 lat0, label, cpu, args.cpu_steps, args.batch, warm=1)
    print(json.dumps({"workload": f"e2e latent step, MOSI shape: batch {args.batch}, vocab "
                                  f"{args.vocab}, T {args.t}, audio {args.a}+2, visual {args.vd}+2",
                      "ms_per_step": {"libmmb_graph": round(ms_graph, 4),
                                      "libmmb_eager_launches": round(ms_hip, 4),
                                      "torch_eager_gpu": round(ms_eager, 4),
                                      "reference_arith_cpu": round(ms_cpu, 2)},
                      "cpu_threads": torch.get_num_threads(),
                      "speedup_vs_eager_gpu": round(ms_eager / ms_graph, 2),
                      "speedup_vs_cpu": round(ms_cpu / ms_graph, 1)}))


if __name__ == "__main__":
    main()
