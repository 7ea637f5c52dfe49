#!/usr/bin/env python3
"""Benchmark of the north-star hot path: SIF + closed-form MMB2 utterance embeddings.

One *step* = one pass of the hot path over a batch of synthetic utterances
already resident in HBM (BASELINE.json configs[3] shape: 40 tokens / frames per
utterance, 3 modalities x 300-d, GloVe-sized V = 400k word table, Zipf(1.1)
ids): for every utterance both its SIF text embedding (weighted average +
first-PC removal, a1-a5) and its closed-form MMB2 embedding (a6-a8) are
produced in device memory.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--utts-per-gpu U]

N > 1 runs one process per GPU (torch.distributed.run, RCCL): each rank owns
its own U utterances (weak scaling: fixed work per GPU) and the ranks
all-reduce the 300x300 Gram once per step — the only collective on the path.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "multimodal-baselines_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
F16_MFMA_PEAK_TFS = 2500.0  # dense f16 MFMA (no sparsity)
F64_MFMA_PEAK_TFS = 78.6  # fp64 MFMA


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def stream_kernel_bytes(L, D, A, Vd):
    """Algorithmic HBM bytes per utterance of mmb_mm2_stream:
    ids + gathered weights + gathered text rows + audio + visual frames (read),
    weighted sum + frame sums + (count, sum w) (write)."""
    return 4 * L + 4 * L + 4 * D * L + 4 * A * L + 4 * Vd * L + 4 * D + 4 * 2 * (D + A + Vd) + 8


def path_bytes(L, D, A, Vd):
    """SURVEY.md §8d B_utt for the whole step (149,120 B at the config-3 shape)."""
    return 4 * L + 4 * L + 4 * D * L + 2 * 4 * A * L + 3 * 4 * D + 4 * D


def cpu_baseline(inp, gen, n_sample):
    """The oracle (CPU restatement of the reference loops + sklearn randomized SVD
    + the MMB2 closed form in fp32 numpy) timed on a bounded sample of the same
    workload, on this host's cores."""
    import numpy as np

    from oracle import mmb2_oracle as M
    from oracle import sif_oracle as O

    import torch

    cores = torch.get_num_threads()  # the BLAS/OpenMP threads actually used (OMP_NUM_THREADS)
    n = n_sample
    table = inp["table"].cpu().numpy()
    wt = inp["wtab"].double().cpu().numpy()
    ids = inp["ids"][:n].long().cpu().numpy()
    audio = inp["audio"][:n].cpu().numpy()
    visual = inp["visual"][:n].cpu().numpy()
    params = M.params_from_module(gen)
    t0 = time.perf_counter()
    w = O.seq2weight_loop(ids, np.ones(ids.shape), wt)          # sif_functions.py:8-15
    emb = O.get_weighted_average(table, ids, w)                  # :28-56
    O.remove_pc(emb, 1)                                          # :58-81
    text = table[ids]
    M.estimate_embedding_overall_gpu2(M.concat_inputs(text, audio, visual), params, w, text,
                                      dtype=np.float32)          # sif2.py:164-208
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "utterance-embeds/s", "cores": cores, "kind": "port",
            "sample": f"{n} utterances of the same workload (L=T={ids.shape[1]}, 3x300-d, "
                      f"V={table.shape[0]}), one pass: oracle/ restatement (python row loops, "
                      f"sklearn-equivalent randomized SVD, numpy BLAS on {cores} threads)",
            "seconds": dt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="synthetic", choices=["synthetic", "pom"],
                    help="synthetic: BASELINE configs[3] (the metric's workload); pom: "
                         "configs[2] shape (V=7763, transcripts padded to 1357, ~370 tokens)")
    ap.add_argument("--utts-per-gpu", type=int, default=None)
    ap.add_argument("--tokens", type=int, default=None)
    ap.add_argument("--vocab", type=int, default=None)
    ap.add_argument("--chunks", type=int, default=None,
                    help="row chunks per step (stream of chunk c+1 overlaps projection of c); "
                         "default 1")
    ap.add_argument("--side-cus", type=int, default=0,
                    help="with --chunks > 1: CUs reserved for the projection + Gram stream")
    ap.add_argument("--side-layout", default="balanced", choices=["balanced", "strided", "high"])
    ap.add_argument("--cpu-sample", type=int, default=8192)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"))
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import mmb_lib
    import models
    import pipeline as P
    import synth

    mmb_lib.require_gpu()
    pom = args.workload == "pom"
    dflt = (10_000, 1357, 7763) if pom else (1_000_000, 40, 400_000)
    U = args.utts_per_gpu or dflt[0]
    T = args.tokens or dflt[1]
    V = args.vocab or dflt[2]
    D = 300
    inp = synth.device_workload(U, T, V, D=D, A=300, Vd=300, seed=1000 + rank, device=dev,
                                mean_len=370.0 if pom else None)
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(D, 300, 300, norm=None).to(dev)

    def allreduce(t):
        if world > 1:
            dist.all_reduce(t)

    step = P.FusedStep(inp, gen.networks(), allreduce=allreduce if world > 1 else None,
                       n_total=U * world, row0=rank * U, chunks=args.chunks,
                       side_cus=args.side_cus, side_layout=args.side_layout)
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        step.run()
    torch.cuda.synchronize()

    # timed region: K steps, barrier + sync on both sides.  HIP events are
    # recorded on the stream each phase is launched on (FusedStep.run trace):
    # the stream kernel's chunks on the caller's stream, projection + Gram of
    # each chunk on the side stream they overlap on.
    assert U * world >= D  # sklearn's direct (non-transposed) randomized-SVD branch
    traces = [dict() for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step.run(trace=traces[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    if int(step.flag.item()) != 0:
        raise RuntimeError("id range flag set")

    names = sorted({n for tr in traces for n in tr})
    phase_ms = {n: sum(a.elapsed_time(b) for tr in traces for a, b in tr.get(n, ()))
                / args.steps for n in names}
    n_launch = sum(len(tr["mm2_stream"]) for tr in traces)
    stream_launch_ms = phase_ms["mm2_stream"] * args.steps / n_launch
    ms_per_step = elapsed * 1e3 / args.steps
    total_utts = U * world * args.steps
    value = total_utts / elapsed

    if rank == 0:
        kb = stream_kernel_bytes(T, D, 300, 300)
        utts_per_launch = U / len(step.bounds)
        achieved = kb * utts_per_launch / (stream_launch_ms / 1e3) / 1e9
        traffic = None
        if os.path.exists(args.traffic_json):
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("utts_per_launch") == utts_per_launch and tj.get("tokens") == T:
                traffic = tj.get("mm2_stream_hbm_bytes_per_launch")
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": ("utt_wave_kernel (mmb_mm2_stream, one wave per utterance)" if T <= 64
                           else "utt_stream_kernel (mmb_mm2_stream, one workgroup per utterance)"),
                "algorithmic_bytes_per_utt": kb, "utts_per_launch": utts_per_launch,
                "avg_launch_ms": round(stream_launch_ms, 4)}
        # MFMA-bound kernels of the step, from their HIP-event phase times:
        # the projection as 3 f16 GEMMs [U, kp] x [kp, ldw] (hi/lo split; its
        # phase includes the fused PC-removal tail), the Gram as the 16x16
        # upper-triangle tiles it computes in fp64
        mfma = {}
        kp, ldw = step.proj.kp, step.proj.ldw
        proj_ms = phase_ms.get("mm2_project+pc_remove", phase_ms.get("mm2_project+gram"))
        if proj_ms and step.s_half:
            tf = 3 * 2 * kp * ldw * U / (proj_ms / 1e3) / 1e12
            mfma["mm2_project_x3b"] = {"bound": "mfma", "achieved": round(tf, 1),
                                       "peak": F16_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                                       "frac": round(tf / F16_MFMA_PEAK_TFS, 4),
                                       "flop_per_utt": 3 * 2 * kp * ldw,
                                       "includes": "fused PC-removal tail"}
        if "gram" in phase_ms:
            nt = (D + 15) // 16
            gflop = nt * (nt + 1) // 2 * 16 * 16 * 2 * U
            tf = gflop / (phase_ms["gram"] / 1e3) / 1e12
            mfma["gram_tri (fp64)"] = {"bound": "mfma", "achieved": round(tf, 2),
                                       "peak": F64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                                       "frac": round(tf / F64_MFMA_PEAK_TFS, 4),
                                       "flop_per_utt": gflop // U}
        pb = path_bytes(T, D, 300, 300)
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            try:
                n_cpu = args.cpu_sample if not pom else max(1, args.cpu_sample * 40 // T)
                cpu = cpu_baseline(inp, gen.cpu(), n_cpu)
            except Exception as exc:  # keep the GPU line even if the host leg fails
                log(f"cpu baseline failed: {exc!r}")
        out = {
            "metric": "utterance-embeds/sec (MMB2, 3 modalities, 300d) at 1/2/4/8 MI355X",
            "value": round(value, 1),
            "unit": "utterance-embeds/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded, generated in HBM; no dataset or checkpoint)",
            "config": {"workload": ("configs[2]: POM-shaped (V=7763, w0=1.0, transcripts padded "
                                    "to 1357, ~370 tokens, aligned frames) x 3 modalities x 300d, "
                                    "SIF(+PC removal) + closed-form MMB2" if pom else
                                    "configs[3]: synthetic utterances x 40 tokens/frames x 3 "
                                    "modalities x 300d, SIF(+PC removal) + closed-form MMB2"),
                       "utts_per_gpu": U, "tokens": T, "vocab": V, "dims": [D, 300, 300],
                       "parallelism": f"dp{world} (utterance shards) + RCCL all-reduce of the "
                                      f"300x300 fp64 Gram"},
            "roofline": roof,
            "path_roofline": {"bytes_per_utt": pb, "achieved": round(pb * U * world / (ms_per_step / 1e3) / world / 1e9, 1),
                              "unit": "GB/s per GPU", "peak": HBM_PEAK_GBS},
            "phase_ms": {k: round(v, 4) for k, v in phase_ms.items()},
            "mfma_rooflines": mfma,
            "chunks": len(step.bounds),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
