#!/usr/bin/env python3
"""Benchmark of the north-star hot path: SIF + closed-form MMB2 utterance embeddings.

One *step* = one pass of the hot path over a batch of synthetic utterances
already resident in HBM (BASELINE.json configs[3] shape: 40 tokens / frames per
utterance, 3 modalities x 300-d, GloVe-sized V = 400k word table, Zipf(1.1)
ids): for every utterance both its SIF text embedding (weighted average +
first-PC removal, a1-a5) and its closed-form MMB2 embedding (a6-a8) are
produced in device memory.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling strong|weak]
                    [--utts U] [--dist-backend nccl|gloo] [--share-device]

Scaling (configs[3]: "1M utterances ... utterance-sharded across 8 x MI355X
... 1/2/4/8-GPU scaling curve"): STRONG by default -- one 1M-utterance split,
rank r owns the contiguous rows distributed.shard_range(1M, N, r) (1M / N
each), generated identically for every N (synth.device_shard: the same word
table on every rank, the utterances from seeded 62.5k-row blocks), so the N
lines of the curve process the same split.  `--scaling weak` (or
--utts-per-gpu) gives every rank its own U rows instead.  The ranks all-reduce
the 300x300 fp64 Gram once per step -- the only collective on the path --
and every rank runs the identical PC solve.  `value` = utterances of the
whole split / the slowest rank's time.

N > 1 runs one process per GPU over RCCL.  Launched without a torchrun
environment (no WORLD_SIZE), `--gpus N` starts the N ranks itself
(torch.distributed.run as a child process, before anything touches the GPU)
and exits with its status.  `--dist-backend gloo --share-device` runs the
same multi-rank branch with every rank on GPU 0 and the collectives on gloo
(the one-GPU test of this branch, tests/test_gpu_bench_dist.py; with
`--dump-rows DIR` each rank saves its PC and a sample of its rows).  Rank 0
prints ONE JSON line.

At N = 1 the line also carries `per_rank_steps` -- the step at the per-rank
sizes of the 2/4/8-GPU strong-scaling runs (500k / 250k / 125k rows of the
same split) -- and `configs_measured`, the other BASELINE configs measured in
the same run: configs[0] (MMB1 text SIF at MOSI shape, GPU and the reference
CPU path), configs[1] (MMB2 at MOSI shape), the ragged configs[3] variant
(Poisson(40) lengths in [1, 64]), configs[2] (POM transcript
length 1357), configs[4] (the regressor's 400-epoch SGD loop at MOSI size)
and the e2e latent step -- plus the fp32-MFMA projection
timed beside the bench path's fp16x3 one, and the CPU baselines.
`--only-main` skips them (profiling passes).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "multimodal-baselines_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
F16_MFMA_PEAK_TFS = 2500.0  # dense f16 MFMA (no sparsity)
F32_MFMA_PEAK_TFS = 157.3  # f32-input MFMA (= the f32 vector rate on gfx950)
F64_MFMA_PEAK_TFS = 78.6  # fp64 MFMA
I8_MFMA_PEAK_TOPS = 5000.0  # dense int8 MFMA (2x f16, no sparsity)
METRIC = "utterance-embeds/sec (MMB2, 3 modalities, 300d) at 1/2/4/8 MI355X"
DTYPE = ("f32 (MMB2 projection: fp16 hi/lo x3 split on the f16 MFMA pipe, fp32 accumulate; "
         "Gram: int8 digits of 30-bit fixed point, exact int32 level sums + f64; "
         "PC solve / removal fp64)")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def stream_kernel_bytes(L, D, A, Vd, text_rows=None):
    """Algorithmic HBM bytes per utterance of mmb_mm2_stream:
    ids + gathered weights + gathered text rows + audio + visual frames (read),
    a2 row + frame sums + (count, sum w) (write).  `text_rows` (mean per
    utterance) overrides L for the text gather: SURVEY §8d counts id-0
    pad/OOV rows once per utterance."""
    tr = L if text_rows is None else text_rows
    return 4 * L + 4 * L + 4 * D * tr + 4 * A * L + 4 * Vd * L + 4 * D + 4 * 2 * (D + A + Vd) + 8


def fused_kernel_bytes(L, D, A, Vd, text_rows=None):
    """Algorithmic HBM bytes per utterance of mmb_mm2_stream_project (the
    stream kernel with the projection fused in): the same reads as
    stream_kernel_bytes; writes the a2 row, the MMB2 row and aux (count,
    sum w, row scale) -- the frame sums never leave the chip."""
    tr = L if text_rows is None else text_rows
    return 4 * L + 4 * L + 4 * D * tr + 4 * A * L + 4 * Vd * L + 4 * D + 4 * D + 12


def path_bytes(L, D, A, Vd, text_rows=None):
    """SURVEY.md §8d B_utt for the whole step (149,120 B at the config-3 shape)."""
    tr = L if text_rows is None else text_rows
    return 4 * L + 4 * L + 4 * D * tr + 4 * (A + Vd) * L + 3 * 4 * D + 4 * D


def host_threads():
    """Host threads the CPU legs use: this process's CPU affinity, capped by an
    OMP_NUM_THREADS the environment sets (the GPU box sets 16, its share of
    a machine whose affinity lists every core)."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    n = min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff
    return n, aff


class cpu_threads:
    """torch and BLAS thread pools set to `n` for a CPU leg, restored after."""

    def __init__(self, n):
        self.n = n

    def __enter__(self):
        import torch
        from threadpoolctl import threadpool_limits

        self.prev = torch.get_num_threads()
        torch.set_num_threads(self.n)
        self.tp = threadpool_limits(self.n)
        return self

    def __exit__(self, *exc):
        import torch

        self.tp.restore_original_limits()
        torch.set_num_threads(self.prev)
        return False


def cpu_baseline(sample, gen, n_sample):
    """The oracle (CPU restatement of the reference loops + sklearn randomized SVD
    + the MMB2 closed form in fp32 numpy) timed on a bounded sample of the same
    workload, on this host's cores."""
    import numpy as np

    from oracle import mmb2_oracle as M
    from oracle import sif_oracle as O

    cores, aff = host_threads()
    table, wt, ids, audio, visual = sample
    params = M.params_from_module(gen)
    with cpu_threads(cores):
        t0 = time.perf_counter()
        w = O.seq2weight_loop(ids, np.ones(ids.shape), wt)          # sif_functions.py:8-15
        emb = O.get_weighted_average(table, ids, w)                  # :28-56
        O.remove_pc(emb, 1)                                          # :58-81
        text = table[ids]
        M.estimate_embedding_overall_gpu2(M.concat_inputs(text, audio, visual), params, w, text,
                                          dtype=np.float32)          # sif2.py:164-208
        dt = time.perf_counter() - t0
    return {"value": round(n_sample / dt, 1), "unit": "utterance-embeds/s", "cores": cores,
            "kind": "port",
            "sample": f"{n_sample} utterances of the same workload (L=T={ids.shape[1]}, 3x300-d, "
                      f"V={table.shape[0]}), one pass of oracle/ (python row loops like the "
                      f"reference, sklearn-equivalent randomized SVD, numpy BLAS)",
            "threads": {"used": cores, "affinity": aff,
                        "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")},
            "sample_note": "bounded to ~10-20 s of host work so the default bench stays within "
                           "minutes (SURVEY §8d suggests 100k utterances: ~2.5 min at this rate)",
            "seconds": round(dt, 3)}


def host_sample(inp, n):
    """Copy the first n utterances of a device workload to the host (before
    the device inputs are freed)."""
    return (inp["table"].cpu().numpy(), inp["wtab"].double().cpu().numpy(),
            inp["ids"][:n].long().cpu().numpy(), inp["audio"][:n].cpu().numpy(),
            inp["visual"][:n].cpu().numpy())


def phase_times(traces, steps):
    names = sorted({n for tr in traces for n in tr})
    return {n: sum(a.elapsed_time(b) for tr in traces for a, b in tr.get(n, ())) / steps
            for n in names}


def load_traffic(name, utts_per_launch, tokens, phase="mm2_stream"):
    """PMC-measured HBM bytes per stream-kernel launch for this exact workload
    and kernel (the fused stream + projection or the plain stream kernel),
    from the committed rocprofv3 summaries (profiles/), never this run."""
    fn = {"synthetic": "traffic_latest.json"}.get(name, f"traffic_{name}_latest.json")
    path = os.path.join(ROOT, "profiles", fn)
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        tj = json.load(f)
    if (tj.get("utts_per_launch") == utts_per_launch and tj.get("tokens") == tokens
            and tj.get("phase", "mm2_stream") == phase):
        sha = f", tree {tj['tree_sha']}" if tj.get("tree_sha") else ""
        return tj.get("mm2_stream_hbm_bytes_per_launch"), f"profiles/{fn} ({tj.get('tag')}{sha})"
    return None, None


# The auxiliary legs (per-rank sizes, the other BASELINE configs) run short
# steps straight after a model build: the chip needs ~25 ms of load to reach
# its clocks (r05 traces: the MOSI step 5.98 -> 5.70 -> 5.46 -> 5.23 -> 5.15
# -> 5.10 -> 5.06 ms over its first steps, the 125k step 3.43 -> 3.11 ms), so
# their warmup runs at least AUX_WARMUP_S of steps beyond its W.  (The main
# timed region keeps exactly W: at 1M rows W = 5 steps is 110 ms.)
AUX_WARMUP_S = 0.1


def run_workload(P, inp, gen, steps, warmup, allreduce=None, world=1, rank=0):
    """FusedStep over `inp`: warmup (W steps, and at least AUX_WARMUP_S of
    them), then `steps` timed steps bracketed by barrier + synchronize, then
    the same number of steps again with HIP events around each phase (the
    per-phase times and the kernels' launch durations; r05: the events are no
    longer inside the timed region, where their ~12 markers per step added to
    the stream).  Returns (step, elapsed_s, per-step traces)."""
    import torch
    import torch.distributed as dist

    U = inp["ids"].shape[0]
    step = P.FusedStep(inp, gen.networks(), allreduce=allreduce, n_total=U * world, row0=rank * U)
    torch.cuda.synchronize()
    w0 = time.perf_counter()
    done = 0
    # (time-based only on one rank: every rank must run the same number of
    # all-reduces)
    while done < warmup or (world == 1 and time.perf_counter() - w0 < AUX_WARMUP_S and done < 1000):
        step.run()
        done += 1
        if done >= warmup:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step.run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    step.check()  # ids in range, no all-zero-weight utterance (one sync, after timing)
    traces = [dict() for _ in range(steps)]
    for k in range(steps):
        step.run(trace=traces[k])
    torch.cuda.synchronize()
    step.check()
    return step, elapsed, traces


def stream_phase(phase_ms):
    """The step's dominant (HBM-bound) phase: the fused stream + projection
    kernel, or the stream kernel of the two-kernel step."""
    for ph in ("mm2_stream_project", "mm2_stream_project_narrow"):
        if ph in phase_ms:
            return ph
    return "mm2_stream"


def stream_roofline(phase_ms, traces, steps, kbytes, U, kernel, traffic_key, T):
    ph = stream_phase(phase_ms)
    n_launch = sum(len(tr[ph]) for tr in traces)
    launch_ms = phase_ms[ph] * steps / n_launch
    achieved = kbytes * U / (launch_ms / 1e3) / 1e9
    traffic, src = load_traffic(traffic_key, U, T, ph)
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_source": (f"rocprofv3 PMC FETCH_SIZE/WRITE_SIZE passes of this workload, "
                               f"{src} -- not measured in this run" if traffic else
                               "no PMC summary of this workload committed"),
            "kernel": kernel, "algorithmic_bytes_per_utt": round(kbytes, 1),
            "utts_per_launch": U, "avg_launch_ms": round(launch_ms, 4),
            "timing": "HIP events on the launch stream around every stream-kernel launch"}


def mfma_rooflines(step, phase_ms, U, D):
    """MFMA-bound kernels of the step on UNPADDED (algorithmic) FLOPs: the
    projection [U, 2(D+A+Vd)] x [.., D+1] as 3 fp16 products (hi/lo split; its
    phase includes the fused PC-removal tail), the Gram's upper triangle in
    fp64 (D(D+1)/2 dot products of U terms)."""
    out = {}
    k_alg = 2 * (step.d + step.a + step.vd)
    if "mm2_stream_project" in phase_ms:
        # the projection runs inside the HBM-bound fused kernel (its own waves,
        # overlapped with the stream): the MFMA rate over the whole kernel
        flop = 3 * 2 * k_alg * (D + 1)
        ms = phase_ms["mm2_stream_project"]
        tf = flop * U / (ms / 1e3) / 1e12
        out["mm2_stream_project (projector waves)"] = {
            "bound": "hbm (the fused kernel)", "achieved": round(tf, 1),
            "peak": F16_MFMA_PEAK_TFS, "unit": "TFLOP/s", "frac": round(tf / F16_MFMA_PEAK_TFS, 4),
            "flop_per_utt": flop, "ms": round(ms, 4),
            "note": "fp16 x3 products issued beside the stream inside one kernel; the kernel is "
                    "HBM-bound, so this is the MFMA work it hides, not a ceiling"}
    if "mm2_stream_project_narrow" in phase_ms:
        k_av = 2 * (step.a + step.vd)
        flop = 3 * 2 * k_av * (D + 1)
        ms = phase_ms["mm2_stream_project_narrow"]
        tf = flop * U / (ms / 1e3) / 1e12
        out["mm2_stream_project_narrow (batch GEMM)"] = {
            "bound": "hbm / latency (the fused kernel)", "achieved": round(tf, 2),
            "peak": F16_MFMA_PEAK_TFS, "unit": "TFLOP/s", "frac": round(tf / F16_MFMA_PEAK_TFS, 5),
            "flop_per_utt": flop, "ms": round(ms, 4),
            "note": "fp16 x3 products of the audio / visual sums (the text rows of the projection "
                    "are applied per word in the text cache) inside the streaming kernel"}
    proj_ms = phase_ms.get("mm2_project+pc_remove", phase_ms.get("mm2_project+gram"))
    if proj_ms and step.s_half:
        flop = 3 * 2 * k_alg * (D + 1)
        tf = flop * U / (proj_ms / 1e3) / 1e12
        out["mm2_project_x3b"] = {"bound": "mfma", "achieved": round(tf, 1),
                                  "peak": F16_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                                  "frac": round(tf / F16_MFMA_PEAK_TFS, 4), "flop_per_utt": flop,
                                  "padded_flop_per_utt": 3 * 2 * step.proj.kp * step.proj.ldw,
                                  "ms": round(proj_ms, 4), "includes": "fused PC-removal tail"}
    if "gram" in phase_ms and getattr(step, "gram_i8", False):
        # 13 int8 digit-pair products of the upper triangle per row (the
        # algorithmic work of the sliced Gram, gram_i8_kernel)
        ops = 13 * D * (D + 1)
        t = ops * U / (phase_ms["gram"] / 1e3) / 1e12
        out["gram_i8 (int8 digits)"] = {"bound": "mfma", "achieved": round(t, 1),
                                        "peak": I8_MFMA_PEAK_TOPS, "unit": "TOP/s",
                                        "frac": round(t / I8_MFMA_PEAK_TOPS, 4), "op_per_utt": ops,
                                        "ms": round(phase_ms["gram"], 4),
                                        "note": "incl. the partial reduction; f64-equivalent "
                                                f"{D * (D + 1) * U / (phase_ms['gram'] / 1e3) / 1e12:.1f} "
                                                "TFLOP/s of G"}
    elif "gram" in phase_ms:
        flop = D * (D + 1)  # 2 * D(D+1)/2 per row
        tf = flop * U / (phase_ms["gram"] / 1e3) / 1e12
        out["gram_tri (fp64)"] = {"bound": "mfma", "achieved": round(tf, 2),
                                  "peak": F64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                                  "frac": round(tf / F64_MFMA_PEAK_TFS, 4), "flop_per_utt": flop,
                                  "ms": round(phase_ms["gram"], 4)}
    return out


def time_fp32_projection(P, step, reps=3):
    """The fp32-MFMA projection (mmb_mm2_project) on the same sums, timed
    beside the bench path's fp16x3 kernel: one extra stream pass writes s in
    fp32, then `reps` projections (HIP events)."""
    import torch

    if not step.s_half:
        return None
    inp = step.inp
    s32 = P.s_buffer(step.n, step.proj.kp, False, step.table.device)
    x, aux = torch.empty_like(step.x), torch.empty((3, step.n), device=step.table.device)
    P.mm2_stream(step.n, step.t, step.d, step.a, step.vd, inp["audio"], inp["visual"],
                 ids32=step.ids, table=step.table, wtab32=inp["wtab"], s_half=False,
                 out=(x, s32, aux))
    out = torch.empty_like(step.mmb2)
    P.mm2_project(s32, x, aux, step.proj, out=out)
    evs = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        P.mm2_project(s32, x, aux, step.proj, out=out)
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    ms = sum(a.elapsed_time(b) for a, b in evs) / reps
    # the fp32 path's rows against the bench path's (both meet the 1e-5 bar in
    # tests/test_gpu_mmb2.py::test_fp16_split_projection_vs_fp32_and_oracle)
    diff = ((out - step.mmb2).abs().amax(1) / step.mmb2.abs().amax(1)).max().item()
    flop = 2 * 2 * (step.d + step.a + step.vd) * (step.d + 1)
    tf = flop * step.n / (ms / 1e3) / 1e12
    del s32, x, aux, out
    return {"ms": round(ms, 4), "achieved": round(tf, 1), "peak": F32_MFMA_PEAK_TFS,
            "unit": "TFLOP/s", "frac": round(tf / F32_MFMA_PEAK_TFS, 4),
            "row_rel_diff_vs_fp16x3": diff,
            "note": "mmb_mm2_project: fp32-input MFMA (exact f32 products), no fused removal"}


def narrow_fused_bytes(L, D, A, Vd):
    """Algorithmic bytes per utterance of mmb_mm2_stream_project_narrow: ids,
    gathered weights, text rows AND their text-cache P rows (4 (D + 4) B,
    L2-resident at MOSI's V), audio and visual frames read; the a2 row, the
    MMB2 row and aux written -- no frame sums leave the chip."""
    return 4 * L + 4 * L + 4 * D * L + 4 * (D + 4) * L + 4 * (A + Vd) * L + 4 * D + 4 * D + 12


def dominant_kernel(step, T, D, text_rows=None):
    """(algorithmic bytes per utterance, name) of the step's HBM-bound kernel."""
    if getattr(step, "narrow_fused", False):
        return (narrow_fused_bytes(T, D, step.a, step.vd),
                "utt_narrow_fused_kernel (mmb_mm2_stream_project_narrow: 8 waves per CU stream "
                "32-utterance batches -- packed frame rows, text rows and their per-word "
                "projections P, the 32 most frequent words from LDS -- then the audio / visual "
                "fp16 x3 GEMM and the row epilogue in the same launch)")
    if step.stream_project:
        return (fused_kernel_bytes(T, D, step.a, step.vd, text_rows=text_rows),
                "utt_fused_kernel (mmb_mm2_stream_project: 4 streaming waves, one per "
                "utterance, two 8-frame load groups in flight, + 4 projecting waves per CU, "
                "sums in an LDS ring)")
    if T > 64:
        kname = "utt_stream_kernel (mmb_mm2_stream, one workgroup per utterance)"
    elif max(step.a, step.vd) <= 128 and step.d > 256:
        kname = ("utt_narrow_kernel (mmb_mm2_stream for narrow frame rows: 2-32 frame rows per "
                 "wave-instruction, one wave per utterance)")
    else:
        kname = "utt_wave_kernel (mmb_mm2_stream, one wave per utterance)"
    return stream_kernel_bytes(T, D, step.a, step.vd, text_rows=text_rows), kname


def stream_uniform_ids(P, step, kbytes, reps=3):
    """The dominant kernel on the same workload with UNIFORM token ids over
    [1, V): every text row a likely L2 / Infinity-Cache miss, so the
    algorithmic-bytes roofline no longer counts Zipf cache hits."""
    import torch

    inp = step.inp
    ids_u = torch.randint(1, step.V, step.ids.shape, dtype=torch.int32, device=step.ids.device)
    if step.stream_project:
        run = lambda: P.mm2_stream_project(step.n, step.t, step.d, step.a, step.vd, inp["audio"],
                                           inp["visual"], step.proj, ids32=ids_u, table=step.table,
                                           wtab32=inp["wtab"], out=(step.x, step.aux, step.mmb2))
    else:
        run = lambda: P.mm2_stream(step.n, step.t, step.d, step.a, step.vd, inp["audio"],
                                   inp["visual"], ids32=ids_u, table=step.table,
                                   wtab32=inp["wtab"], s_half=True, out=(step.x, step.s, step.aux))
    run()
    evs = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        run()
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    ms = sum(a.elapsed_time(b) for a, b in evs) / reps
    ach = kbytes * step.n / (ms / 1e3) / 1e9
    del ids_u
    return {"avg_launch_ms": round(ms, 4), "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
            "note": "same frames and table, token ids uniform over [1, V) instead of Zipf(1.1)"}


def two_kernel_step(P, step, gen, steps=5, warmup=1):
    """The same workload through the two-kernel step (mmb_mm2_stream writes the
    sums s to HBM, mmb_mm2_project_x3_rmpc reads them back and fuses the PC
    removal), timed beside the fused default: the A/B of the fusion."""
    import torch

    two = P.FusedStep(step.inp, gen.networks(), stream_project=False)
    for _ in range(warmup):
        two.run()
    traces = [dict() for _ in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        two.run(trace=traces[k])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ph = phase_times(traces, steps)
    diff = ((two.mmb2 - step.mmb2).abs().amax(1) / step.mmb2.abs().amax(1)).max().item()
    out = {"ms_per_step": round(el * 1e3 / steps, 4), "value": round(step.n * steps / el, 1),
           "phase_ms": {k: round(v, 4) for k, v in ph.items()},
           "mmb2_row_rel_diff_vs_fused": diff,
           "note": "mmb_mm2_stream -> s (fp16 hi/lo, 7.3 KB per utterance) in HBM -> "
                   "mmb_mm2_project_x3_rmpc; same Gram / PC solve"}
    del two
    torch.cuda.empty_cache()
    return out


def ragged_config(P, models, synth, dev, steps, warmup, U):
    """SURVEY §8d's second configs[3] run: Poisson(40) lengths clipped to
    [1, 64], padded with id 0 (weight 1.0) and -10 frames, T = 64."""
    import torch

    T, V, D = 64, 400_000, 300
    inp = synth.device_workload(U, T, V, D=D, A=300, Vd=300, seed=2000, device=dev,
                                poisson_len=40.0)
    lens = inp.pop("lengths")
    ids = inp["ids"]
    nz = (ids != 0).sum().item() / U
    any0 = (ids == 0).any(1).float().mean().item()
    mean_len = lens.float().mean().item()
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(D, 300, 300, norm=None).to(dev)
    step, elapsed, traces = run_workload(P, inp, gen, steps, warmup)
    ph = phase_times(traces, steps)
    kb, kname = dominant_kernel(step, T, D, text_rows=nz + any0)
    roof = stream_roofline(ph, traces, steps, kb, U, kname + ", T = 64", "ragged", T)
    pb = path_bytes(T, D, 300, 300, text_rows=nz + any0)
    out = {"workload": "configs[3] ragged: Poisson(40) lengths clipped to [1, 64], padded to 64 "
                       "with id 0 (w0 = 1.0) and -10 frames, V = 400k, Zipf(1.1) ids, 3 x 300-d",
           "utts": U, "tokens": T, "mean_len": round(mean_len, 3),
           "value": round(U * steps / elapsed, 1), "unit": "utterance-embeds/s",
           "ms_per_step": round(elapsed * 1e3 / steps, 4), "roofline": roof,
           "path_roofline": {"bytes_per_utt": round(pb, 1),
                             "achieved": round(pb * U / (elapsed / steps) / 1e9, 1),
                             "unit": "GB/s", "peak": HBM_PEAK_GBS},
           "phase_ms": {k: round(v, 4) for k, v in ph.items()},
           "text_rows_per_utt": round(nz + any0, 3)}
    del step, inp
    return out


def pom_config(P, models, synth, dev, steps, warmup, U=10_000):
    """configs[2]: POM transcript length (padded to 1357 like pom_test_ids.npy,
    ~370 tokens, V = 7763, w0 = 1.0), aligned 300-d frames."""
    import torch

    T, V, D = 1357, 7763, 300
    inp = synth.device_workload(U, T, V, D=D, A=300, Vd=300, seed=3000, device=dev,
                                mean_len=370.0)
    inp.pop("lengths", None)
    ids = inp["ids"]
    nz = (ids != 0).sum().item() / U
    any0 = (ids == 0).any(1).float().mean().item()
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(D, 300, 300, norm=None).to(dev)
    step, elapsed, traces = run_workload(P, inp, gen, steps, warmup)
    ph = phase_times(traces, steps)
    # the workgroup kernel loads every token's row (pads and OOV hit one cached
    # row); algorithmic bytes count the id-0 row once
    kb = stream_kernel_bytes(T, D, 300, 300, text_rows=nz + any0)
    roof = stream_roofline(ph, traces, steps, kb, U, "utt_stream_kernel (one 320-thread "
                           "workgroup per utterance, 512-token LDS chunks)", "pom", T)
    out = {"workload": "configs[2] POM-shaped: V = 7763, w0 = 1.0, transcripts padded to 1357 "
                       "(~370 tokens), aligned 300-d audio/visual frames (-10 pads)",
           "utts": U, "tokens": T, "value": round(U * steps / elapsed, 1),
           "unit": "utterance-embeds/s", "ms_per_step": round(elapsed * 1e3 / steps, 4),
           "roofline": roof, "phase_ms": {k: round(v, 4) for k, v in ph.items()},
           "text_rows_per_utt": round(nz + any0, 3)}
    del step, inp
    return out


def regressor_config(dev, cpu_epochs=40):
    """configs[4]: the sentiment regressor's training loop at MOSI size
    (1284 / 229 / 686 rows, H = 100, n_out = 1, batch 32, SGD lr 0.1, 400
    epochs, validation every 10 epochs, sentiment_model.py:76-163) through the
    product's train_sentiment, plus the pure kernel (all 16,400 SGD steps in one
    mmb_mlp_train launch) and the CPU restatement on a sample of epochs."""
    import contextlib
    import io

    import numpy as np
    import torch
    from torch.utils.data import DataLoader

    import mmb_lib as L
    import sentiment_model as SM
    from oracle import regressor_oracle as R

    sizes, H, epochs, B, lr = (1284, 229, 686), 100, 400, 32, 0.1
    rng = np.random.default_rng(7)
    lat = [(rng.standard_normal((n, 300)) / np.sqrt(300)).astype(np.float32) for n in sizes]
    wp = rng.standard_normal(300).astype(np.float32) * 2
    lab = [np.clip(l @ wp + 0.9 * rng.standard_normal(len(l)), -3, 3).astype(np.float32)
           for l in lat]
    args = {"sentiment_hidden_size": H, "n_sentiment_epochs": epochs, "sentiment_lr": lr,
            "early_stopping": False, "dataset": "mosi", "lr_decay": 0.5}
    steps = epochs * ((sizes[0] + B - 1) // B)

    # (1) the product loop (host early-stopping logic, a validation + host sync
    # every 10 epochs, mmb_mlp_train per block of epochs)
    def product_run():
        torch.manual_seed(11)
        model = SM.SentimentModel(300, H, 1).to(dev)
        tr = DataLoader(SM.SentimentData(lab[0], dev), batch_size=B, shuffle=True)
        va = DataLoader(SM.SentimentData(lab[1], dev), batch_size=B, shuffle=True)
        tl, vl = (torch.tensor(l, device=dev) for l in lat[:2])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            SM.train_sentiment(args, model, tr, tl, va, vl, None)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    product_run()  # warm-up (module load, first launches)
    t_prod = min(product_run() for _ in range(2))

    # (2) the kernel alone: one launch, every step of the 400 epochs
    torch.manual_seed(11)
    model = SM.SentimentModel(300, H, 1).to(dev)
    w1, b1, w2, b2 = (p.detach() for p in (model.hidden1.weight, model.hidden1.bias,
                                             model.out.weight, model.out.bias))
    x = torch.tensor(lat[0], device=dev)
    y = torch.tensor(lab[0], device=dev).reshape(-1, 1).contiguous()
    perm = torch.cat([torch.randperm(sizes[0]) for _ in range(epochs)]).to(dev)
    sl = torch.empty(steps, device=dev)
    ws = torch.zeros(L.query("mmb_mlp_workspace_bytes", 300, H) // 4 + 4, device=dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    L.call("mmb_mlp_train", L.ptr(x), L.ptr(y), L.ptr(perm), sizes[0], epochs, B, 300, H, 1,
           float(lr), L.ptr(w1), L.ptr(b1), L.ptr(w2), L.ptr(b2), L.ptr(sl), None, None, None, 0,
           1, 0, None, L.ptr(ws), None, L.stream_ptr())
    b.record()
    torch.cuda.synchronize()
    k_ms = a.elapsed_time(b)
    flop_step = 2 * B * 300 * H * 2 + 2 * B * H * 1 * 3  # fwd + dW1 GEMMs (+ the O=1 head)
    tf = flop_step * steps / (k_ms / 1e3) / 1e12

    # (3) the CPU restatement of the reference loop (torch CPU, its own RNG
    # order), a sample of epochs
    cores, aff = host_threads()
    with cpu_threads(cores):
        cargs = dict(args, n_sentiment_epochs=cpu_epochs)
        torch.manual_seed(11)
        m = R.Regressor(300, H, 1)
        loaders = [DataLoader(R._Labels(l), batch_size=B, shuffle=True) for l in lab[:2]]
        t0 = time.perf_counter()
        R.train(cargs, m, loaders[0], torch.tensor(lat[0]), loaders[1], torch.tensor(lat[1]))
        t_cpu = time.perf_counter() - t0
    cpu_steps = cpu_epochs * ((sizes[0] + B - 1) // B)
    return {"workload": "configs[4]: regressor 300 -> 100 -> 1 on MOSI-sized splits 1284 / 229 / "
                        "686, batch 32, SGD lr 0.1, 400 epochs, validation every 10 epochs",
            "steps": steps, "train_s": round(t_prod, 4),
            "ms_per_step": round(t_prod * 1e3 / steps, 5),
            "kernel": {"name": "mlp_train_mc_kernel (mmb_mlp_train: every SGD step in one launch "
                               "of ceil(H / 32) workgroups, one hidden tile each, one exchange of "
                               "output shares per step)",
                       "ms_400_epochs": round(k_ms, 3), "us_per_step": round(k_ms * 1e3 / steps, 3),
                       "mfma": {"achieved": round(tf, 3), "peak": F32_MFMA_PEAK_TFS,
                                "unit": "TFLOP/s", "frac": round(tf / F32_MFMA_PEAK_TFS, 5),
                                "flop_per_step": flop_step,
                                "bound": "latency: 16,400 dependent SGD steps in sequence, "
                                         "each a forward, an exchange between the workgroups "
                                         "and a backward (~1 us of MFMA per workgroup)"}},
            "cpu_baseline": {"ms_per_step": round(t_cpu * 1e3 / cpu_steps, 4),
                             "train_s_400_epochs_extrapolated": round(t_cpu * epochs / cpu_epochs, 2),
                             "cores": cores, "kind": "port",
                             "sample": f"{cpu_epochs} of 400 epochs of oracle/regressor_oracle.py "
                                       f"(torch CPU, the reference's per-batch loop)"},
            "speedup_vs_cpu": round((t_cpu / cpu_steps) / (t_prod / steps), 1)}


def self_launch(n, argv):
    """`bench.py --gpus N` outside torchrun: start N ranks as a child
    torch.distributed.run (this process has not touched the GPU) and return
    its exit status.  The ranks inherit this environment (incl.
    HSA_ENABLE_IPC_MODE_LEGACY=0 for RCCL's dmabuf IPC)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    log(f"bench: launching {n} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd, env=env)


def launch_check():
    """--launch-check: every rank joins the process group (gloo without a
    GPU) and all-reduces a one; rank 0 prints the ranks it saw."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.ones(1)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"launch_check": True, "ranks_seen": world,
                          "allreduce_sum": int(t.item()), "pid": os.getpid()}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def per_rank_steps(P, inp, gen, steps, warmup, sizes):
    """The step on the first U rows of the split, for U = the per-rank sizes
    of the strong-scaling curve (1M / N): the curve each rank follows, minus
    the all-reduce (720 KB over xGMI) and the rank skew, which one GPU cannot
    show."""
    import torch

    out = {}
    for u in sizes:
        sl = {k: (v[:u] if k in ("ids", "audio", "visual") else v) for k, v in inp.items()}
        step, elapsed, traces = run_workload(P, sl, gen, steps, warmup)
        ph = phase_times(traces, steps)
        out[str(u)] = {"utts": u, "ms_per_step": round(elapsed * 1e3 / steps, 4),
                       "value": round(u * steps / elapsed, 1),
                       "phase_ms": {k: round(v, 4) for k, v in ph.items()}}
        del step
        torch.cuda.empty_cache()
    return out


def table_resident_roofline(roof, kb, U, D, T, narrow_fused=False):
    """configs[1] (MOSI shape): the 3.6 MB word table (and the narrow fused
    kernel's 3.7 MB text cache) is L2 / Infinity-Cache resident (its rows are
    24 KB -- 48 KB with the P rows -- of the bytes per utterance), so on all
    algorithmic bytes the stream kernel runs above the HBM peak.  The HBM
    roofline is restated in place on the bytes HBM must deliver (text rows
    excluded); the all-bytes rate is kept beside it as *_incl_table."""
    hbm_b = kb - 4 * D * T - (4 * (D + 4) * T if narrow_fused else 0)
    hbm_ach = hbm_b * U / (roof["avg_launch_ms"] / 1e3) / 1e9
    roof.update({"achieved_incl_table": roof["achieved"], "frac_incl_table": roof["frac"],
                 "algorithmic_bytes_per_utt_incl_table": roof["algorithmic_bytes_per_utt"],
                 "achieved": round(hbm_ach, 1), "frac": round(hbm_ach / HBM_PEAK_GBS, 4),
                 "algorithmic_bytes_per_utt": hbm_b,
                 "bytes_note": "achieved / frac on the HBM bytes (ids, weights, frames read; a2 "
                               "row and aux written, and the frame sums (two-kernel step) or the "
                               "MMB2 row (narrow fused kernel)); the word-table and text-cache "
                               "rows come from L2 / Infinity Cache (*_incl_table counts them)"})
    return roof


def _lat_ms(fn, dev, reps):
    """Host wall per call (each call ends with a device sync): median, min."""
    import statistics

    import torch

    ts = []
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        ts.append((time.perf_counter() - t0) * 1e3)
    return round(statistics.median(ts), 4), round(min(ts), 4)


def dataset_splits_config(P, models, synth, dev, reps=30):
    """configs[0]/[1]/[2] at their real sizes and call pattern: SIF (+ its own
    PC) and MMB2 once per split (simplesif.py:296-311; --time_test :862-880).
    MOSI: train / valid / test = 1284 / 229 / 686 utterances, T = 20, A = 76,
    Vd = 48 (synthetic: the MOSI h5 is absent).  POM: the reference's own
    pom_valid_ids (100 x 1089) / pom_test_ids (203 x 1357) and
    pom_word_weights.npy (tests/golden/g11_pom_splits.npz), V = 7763, aligned
    300-d frames.  Per split: eager (FusedStep.run + its flag check), one HIP
    graph replay per split (StepGraph), and all splits of a dataset in ONE
    graph with concurrent branches (the splits' PC solves side by side).  Every
    time is host wall around the call including the sync that reads the flag
    (what a CLI user waits for), median of `reps`; phase_ms: HIP events of an
    eager run queued behind a device sleep (the host ahead of the GPU: GPU time
    per phase), phase_ms_host_bound: the same events with the launches issued
    as the host gets to them (the GPU idles between phases).  SIF rows of the POM splits against the reference's recorded
    rows (g11)."""
    import numpy as np
    import torch

    from oracle import mmb2_oracle as M

    z = np.load(os.path.join(ROOT, "tests", "golden", "g11_pom_splits.npz"), allow_pickle=False)
    sets = {"mosi": (synth.mosi_splits(), ("train", "valid", "test"), 76, 48),
            "pom": (synth.pom_splits(z["valid_ids"], z["test_ids"], z["weights"],
                                     int(z["table_seed"])), ("valid", "test"), 300, 300)}
    out = {}
    for name, (splits, names, A, Vd) in sets.items():
        torch.manual_seed(0)
        gen = models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(dev)
        inps = [synth.to_device(sp, dev) for sp in splits]
        steps = [P.FusedStep(inp, gen.networks()) for inp in inps]
        res = {"splits": {}}
        for nm, sp, st in zip(names, splits, steps):
            st.run(check=True)
            tr = {}
            st.run(trace=tr)  # launched as the host gets to them: the GPU waits between
            torch.cuda.synchronize(dev)
            ph_host = {k: round(sum(a.elapsed_time(b) for a, b in v), 4) for k, v in tr.items()}
            # the same launches queued behind a device sleep, so the host is
            # ahead and each phase's events bracket GPU work only
            tr = {}
            torch.cuda._sleep(5_000_000)
            st.run(trace=tr)
            torch.cuda.synchronize(dev)
            ph = {k: round(sum(a.elapsed_time(b) for a, b in v), 4) for k, v in tr.items()}
            eager = _lat_ms(lambda: st.run(check=True), dev, reps)
            g = P.StepGraph(st)
            graph = _lat_ms(lambda: g.run(check=True), dev, reps)
            n, L = sp["ids"].shape
            res["splits"][nm] = {"utts": n, "tokens": L, "eager_ms": eager[0],
                                 "graph_ms": graph[0], "graph_ms_min": graph[1],
                                 "phase_ms": ph, "kernel_ms": round(sum(ph.values()), 4),
                                 "phase_ms_host_bound": ph_host}
            if name == "pom":
                got = st.sif.double().cpu().numpy()[::int(z["row_step"])]
                res["splits"][nm]["sif_row_rel_err_vs_reference"] = float(
                    M.row_rel_err(got, z[f"{nm}_out_rows"]))
            del g
        gall = P.StepGraph(steps, concurrent=True)
        allm = _lat_ms(lambda: gall.run(check=True), dev, reps)
        gser = P.StepGraph(steps, concurrent=False)
        serm = _lat_ms(lambda: gser.run(check=True), dev, reps)
        res["all_splits_one_graph_concurrent_ms"] = allm[0]
        res["all_splits_one_graph_serial_ms"] = serm[0]
        res["per_split_ms_concurrent_graph"] = round(allm[0] / len(steps), 4)
        res["utterances"] = int(sum(sp["ids"].shape[0] for sp in splits))
        res["value_concurrent_graph"] = round(res["utterances"] / (allm[0] / 1e3), 1)
        res["unit"] = "utterance-embeds/s (SIF + MMB2, every split with its own PC)"
        out[name] = res
        del gall, gser, steps, inps
        torch.cuda.empty_cache()
    out["note"] = ("host wall per call incl. the flag check's sync; graph-replay floor per "
                   "the MI355X guide ~10-16 us per replay")
    return out


def mosi_mmb2_config(P, models, synth, dev, steps, warmup, U=1_000_000):
    """configs[1]: MMB2 at MOSI shape -- T = 20 aligned frames, COVAREP 74 + 2
    positional dims = 76, FACET 46 + 2 = 48 (make_configs.py:28),
    V = 3016 (sif_functions.py:48) -- on 1M synthetic utterances, the step
    FusedStep picks for these frame widths (pipeline.fused_pays: the
    two-kernel step, stream kernel + projection, 1.5x the fused kernel's rate
    at 76 / 48-float frames).  The 3.6 MB word table sits in L2 / Infinity
    Cache, so the roofline is given on algorithmic bytes (text rows counted)
    and on the bytes that must come from HBM (text rows excluded)."""
    import torch

    T, V, D, A, Vd = 20, 3016, 300, 76, 48
    inp = synth.device_workload(U, T, V, D=D, A=A, Vd=Vd, seed=4000, device=dev)
    torch.manual_seed(0)
    g = models.AudioVisualGeneratorMultimodal(D, A, Vd, norm=None).to(dev)
    step, elapsed, traces = run_workload(P, inp, g, steps, warmup)
    ph = phase_times(traces, steps)
    kb, kname = dominant_kernel(step, T, D)
    roof = stream_roofline(ph, traces, steps, kb, U, kname + f", T = {T}, A = {A}, Vd = {Vd}",
                           "mosi", T)
    table_resident_roofline(roof, kb, U, D, T, narrow_fused=step.narrow_fused)
    out = {"workload": f"configs[1] MOSI-shaped: T = {T}, A = {A} (COVAREP 74 + 2 pos), Vd = {Vd} "
                       f"(FACET 46 + 2 pos), V = {V}, Zipf(1.1) ids, U(-1, 1) frames, SIF(+PC "
                       "removal) + closed-form MMB2",
           "utts": U, "value": round(U * steps / elapsed, 1), "unit": "utterance-embeds/s",
           "ms_per_step": round(elapsed * 1e3 / steps, 4), "roofline": roof,
           "phase_ms": {k: round(v, 4) for k, v in ph.items()}}
    n_cpu = 20_000
    sample = host_sample(inp, n_cpu)
    gen_cpu = models.AudioVisualGeneratorMultimodal(D, A, Vd, norm=None)
    gen_cpu.load_state_dict({k: v.cpu() for k, v in g.state_dict().items()})
    del step, inp
    torch.cuda.empty_cache()
    try:
        out["cpu_baseline"] = cpu_baseline(sample, gen_cpu, n_cpu)
    except Exception as exc:  # keep the GPU numbers if the host leg fails
        out["cpu_baseline"] = {"error": repr(exc)}
    return out


def mmb1_sif_mosi_config(dev, reps=50):
    """configs[0]: MMB1 text-only SIF (--unimodal) at MOSI shape -- N = 2199
    utterances (1284 + 229 + 686, one split-sized batch), L = 20, V = 3016 --
    a1-a5 on the GPU (pipeline.sif_embeddings: device-resident inputs, one
    launch chain + the flag check's sync) against the reference's CPU path
    restated in oracle/ (its seq2weight / get_weighted_average row loops and
    sklearn's TruncatedSVD, sif.py:84-94 -> sif_functions.py:8-96) on the
    host cores, same inputs, results compared."""
    import numpy as np
    import torch

    import pipeline as P
    import synth
    from oracle import mmb2_oracle as M
    from oracle import sif_oracle as O

    N, L, V = 2199, 20, 3016
    E = synth.word_table(V, 300, seed=21)
    wt = synth.sif_weights(V, w0=0.0)
    ids = synth.token_ids(N, L, V, seed=22, ragged=True)
    table = torch.tensor(E, device=dev)
    wt32 = torch.tensor(wt, device=dev, dtype=torch.float32)
    ids32 = torch.as_tensor(ids, dtype=torch.int32, device=dev)
    out, _ = P.sif_embeddings(table, ids32, wtab32=wt32)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out, _ = P.sif_embeddings(table, ids32, wtab32=wt32)
    torch.cuda.synchronize()
    gpu_s = (time.perf_counter() - t0) / reps
    cores, aff = host_threads()
    with cpu_threads(cores):
        t0 = time.perf_counter()
        ref = O.get_sentence_embeddings(E, wt, ids)
        cpu_s = time.perf_counter() - t0
    err = M.row_rel_err(out.cpu().numpy(), ref)
    return {"workload": f"configs[0] MMB1 text SIF at MOSI shape: N = {N}, L = {L}, V = {V}, "
                        "ragged ids (id-0 pads, w0 = 0)",
            "gpu": {"ms_per_call": round(gpu_s * 1e3, 4), "value": round(N / gpu_s, 1),
                    "unit": "utterance-embeds/s",
                    "note": "pipeline.sif_embeddings on device-resident inputs (a1-a5, PC over "
                            "the batch), incl. the flag / finite-PC check's host sync"},
            "cpu_baseline": {"ms_per_call": round(cpu_s * 1e3, 3), "value": round(N / cpu_s, 1),
                             "cores": cores, "kind": "port",
                             "sample": "the whole batch through oracle/sif_oracle."
                                       "get_sentence_embeddings (the reference's loops + sklearn "
                                       "TruncatedSVD)"},
            "row_rel_err_vs_cpu": err, "speedup_vs_cpu": round(cpu_s / gpu_s, 1)}


def latent_step_config(dev, steps=50, cpu_steps=3):
    """one e2e latent-optimisation step at MOSI shape
    (batch 64, V = 3016, T = 20; simplesif.py:712-790: generator forward, word
    + Gaussian objective, regressor, backward, SGD) -- the CLI's default (HIP
    graph of the step's device work, tools/latent_bench.py), the same kernels
    launched eagerly, the reference's torch arithmetic on the GPU and on the
    host cores -- plus word_zsum_kernel (the [B, V] cosine / acos objective
    on fp32 MFMA, losses.py:68-95) timed alone with HIP events."""
    import copy

    import torch

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import latent as LT
    import latent_bench as LB

    class A:
        n, t, vocab, a, vd, batch = 1284, 20, 3016, 75, 46, 64

    args = A()
    cfg, obj, gen, senti, lat0, label, data = LB.build(args, dev)
    ms_graph = LB.run(cfg, None, copy.deepcopy(gen), copy.deepcopy(senti), lat0, label, dev,
                      steps, args.batch, graph_obj=obj)
    ms_eager = LB.run(cfg, obj.log_prob, copy.deepcopy(gen), copy.deepcopy(senti), lat0, label,
                      dev, steps, args.batch)
    # the reference's arithmetic on the GPU: torch's LayerNorm and regressor
    # (no libmmb kernel in this leg)
    ms_torch = LB.run(cfg, LB.eager_objective(cfg, data, dev), LB.plain_torch(gen).float(),
                      LB.CpuSenti(senti), lat0, label, dev, steps, args.batch)
    # the word objective's forward kernel alone: B = 64 latents x V = 3016 words
    lat = (torch.randn(args.batch, 300, device=dev) * 0.5)
    j = torch.arange(args.batch, device=dev)
    wfn = lambda: LT.word_log_prob(lat, obj.table, obj.w[j], obj.m[j], 1e-3, ids=obj.ids[j])
    wfn()
    evs = []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        wfn()
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    w_ms = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
    flop = 2 * args.batch * args.vocab * 304 * 2  # C = Wn U^T and G += R Wn (K = 304)
    tf = flop / (w_ms / 1e3) / 1e12
    cores, aff = host_threads()
    with cpu_threads(cores):
        cpu = torch.device("cpu")
        ms_cpu = LB.run(cfg, LB.eager_objective(cfg, data, cpu), LB.plain_torch(gen).cpu(),
                        LB.CpuSenti(senti), lat0, label, cpu, cpu_steps, args.batch, warm=1)
    return {"workload": "e2e latent step at MOSI shape: batch 64, V = 3016, T = 20, audio 75+2, "
                        "visual 46+2 (simplesif.py:712-790)",
            "ms_per_step": {"libmmb_graph": round(ms_graph, 4),
                            "libmmb_eager_launches": round(ms_eager, 4),
                            "torch_reference_arith_gpu": round(ms_torch, 4),
                            "reference_arith_cpu": round(ms_cpu, 2)},
            "word_forward": {"kernel": "word_zsum_kernel + word_finish_kernel "
                                       "(mmb_word_logprob_fwd: fp32 MFMA 16x16x4)",
                             "ms": round(w_ms, 5), "flop": flop, "achieved": round(tf, 3),
                             "peak": F32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                             "frac": round(tf / F32_MFMA_PEAK_TFS, 5),
                             "bound": "latency: 0.24 GFLOP over 4 x 189 workgroups, a few us"},
            "cpu_baseline": {"ms_per_step": round(ms_cpu, 2), "cores": cores, "kind": "port",
                             "sample": f"{cpu_steps} steps of the reference's torch arithmetic "
                                       "(oracle/latent_oracle) on the host"},
            "speedup_vs_torch_gpu": round(ms_torch / ms_graph, 2),
            "speedup_vs_cpu": round(ms_cpu / ms_graph, 1)}


def hbm_ceilings(dev, nbytes=4 << 30, reps=10):
    """Same-process HBM ceilings (SURVEY §8d "a measured stream-copy
    ceiling"): libmmb's float4 probes (non-temporal, 4 loads in flight per
    lane) over `nbytes` -- far above the 256 MB Infinity Cache -- timed with
    HIP events on the launch stream, best of a few grid sizes.  Copy counts
    read + write bytes."""
    import torch

    import mmb_lib as L

    src = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).uniform_()
    dst = torch.empty_like(src)
    cus = L.cu_count(dev)
    sink = torch.empty(cus * 16, dtype=torch.int32, device=dev)
    sp = L.stream_ptr()
    out = {}
    for name, launch, moved in (
            ("copy", lambda b, nt: L.call("mmb_probe_copy", L.ptr(src), L.ptr(dst), nbytes, b, nt,
                                          sp), 2 * nbytes),
            ("read", lambda b, nt: L.call("mmb_probe_read", L.ptr(src), nbytes, b, nt,
                                          L.ptr(sink), sp), nbytes)):
        best, how = 0.0, None
        for nt in (0, 1):
            for per_cu in (1, 2, 4, 8):
                b = cus * per_cu
                launch(b, nt)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    launch(b, nt)
                e1.record()
                torch.cuda.synchronize()
                r = moved * reps / (e0.elapsed_time(e1) / 1e3) / 1e9
                out.setdefault("sweep", {})[f"{name}_nt{nt}_wg{per_cu}"] = round(r, 1)
                if r > best:
                    best, how = r, f"nt={nt}, {per_cu} workgroups per CU"
        out[name] = round(best, 1)
        out[name + "_config"] = how
    del src, dst, sink
    torch.cuda.empty_cache()
    return out


def annotate_ceilings(obj, ceil):
    """Every GB/s roofline in the line gains the measured ceilings beside the
    8 TB/s spec: copy_ceiling_gbs / read_ceiling_gbs and achieved over each."""
    if isinstance(obj, dict):
        if (str(obj.get("unit", "")).startswith("GB/s") and isinstance(obj.get("achieved"),
                                                                      (int, float))):
            obj["copy_ceiling_gbs"] = ceil["copy"]
            obj["read_ceiling_gbs"] = ceil["read"]
            obj["frac_of_ceiling"] = round(obj["achieved"] / ceil["copy"], 4)
            obj["frac_of_read_ceiling"] = round(obj["achieved"] / ceil["read"], 4)
        for v in obj.values():
            annotate_ceilings(v, ceil)
    elif isinstance(obj, list):
        for v in obj:
            annotate_ceilings(v, ceil)


def dump_rows(path, rank, row0, step):
    """--dump-rows: this rank's PC and every 97th of its SIF / MMB2 rows (plus
    its last), for tests/test_gpu_bench_dist.py to compare with the unsharded
    step."""
    import numpy as np
    import torch

    os.makedirs(path, exist_ok=True)
    n = step.n
    idx = torch.tensor(sorted(set(range(0, n, 97)) | {n - 1}), device=step.sif.device)
    np.savez(os.path.join(path, f"rank{rank}.npz"), row0=row0, n=n, pc=step.pc.cpu().numpy(),
             idx=idx.cpu().numpy(), sif=step.sif[idx].cpu().numpy(),
             mmb2=step.mmb2[idx].cpu().numpy(), flag=int(step.flag.item()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="synthetic", choices=["synthetic", "pom", "ragged", "mosi"],
                    help="synthetic: BASELINE configs[3] (the metric's workload); pom: configs[2] "
                         "shape (V=7763, transcripts padded to 1357, ~370 tokens); ragged: "
                         "configs[3] with Poisson(40) lengths in [1, 64]; mosi: configs[1] shape "
                         "(T = 20, A = 76, Vd = 48, V = 3016; also in configs_measured)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default=None,
                    help="strong (default): one split of --utts utterances sharded over the "
                         "ranks; weak: --utts (or --utts-per-gpu) utterances per rank")
    ap.add_argument("--utts", type=int, default=None,
                    help="utterances of the split (strong) or per rank (weak); default 1M "
                         "(POM: 10k)")
    ap.add_argument("--utts-per-gpu", type=int, default=None,
                    help="utterances per rank; implies --scaling weak (at N = 1 the same as --utts)")
    ap.add_argument("--tokens", type=int, default=None)
    ap.add_argument("--vocab", type=int, default=None)
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL over xGMI (the product); gloo: the collectives on the host "
                         "(with --share-device: the multi-rank branch on one GPU)")
    ap.add_argument("--share-device", action="store_true",
                    help="every rank on GPU 0 (tests of the N > 1 branch on a one-GPU box)")
    ap.add_argument("--dump-rows", default=None,
                    help="directory: each rank saves its PC and a sample of its rows")
    ap.add_argument("--chunks", type=int, default=None,
                    help="row chunks per step (stream of chunk c+1 overlaps projection of c); "
                         "default 1")
    ap.add_argument("--side-cus", type=int, default=0,
                    help="with --chunks > 1: CUs reserved for the projection + Gram stream")
    ap.add_argument("--side-layout", default="balanced", choices=["balanced", "strided", "high"])
    ap.add_argument("--cpu-sample", type=int, default=8192)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--only-main", action="store_true",
                    help="skip per_rank_steps, configs_measured (the other BASELINE configs) and "
                         "the fp32 projection timing")
    ap.add_argument("--only-leg", default=None,
                    help="run only this configs_measured leg (e.g. dataset_splits) and print it")
    ap.add_argument("--launch-check", action="store_true",
                    help="only start the ranks and all-reduce a one (tests the launcher)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if not args.launch_check and not args.share_device:
            import torch  # device_count() does not initialise the GPU

            have = torch.cuda.device_count()
            if have < args.gpus:
                log(f"bench: --gpus {args.gpus} but only {have} GPU(s) visible")
                return 2
        return self_launch(args.gpus, sys.argv[1:])
    if args.launch_check:
        return launch_check()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.share_device else int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        ranks_seen = dist.get_world_size()
        one = torch.ones(1, device=dev)
        dist.all_reduce(one)  # every rank is live on the backend before the timed steps
        assert int(one.item()) == ranks_seen == world
    else:
        ranks_seen = 1

    import distributed as Dist
    import mmb_lib
    import models
    import pipeline as P
    import synth

    mmb_lib.require_gpu()
    if args.only_leg:
        legs = {"dataset_splits": lambda: dataset_splits_config(P, models, synth, dev),
                "mosi_mmb2": lambda: mosi_mmb2_config(P, models, synth, dev, 5, 2),
                "regressor": lambda: regressor_config(dev),
                "latent_step": lambda: latent_step_config(dev),
                "mmb1_sif_mosi": lambda: mmb1_sif_mosi_config(dev)}
        print(json.dumps({args.only_leg: legs[args.only_leg]()}), flush=True)
        return 0
    kind = args.workload
    dflt = {"synthetic": (1_000_000, 40, 400_000), "pom": (10_000, 1357, 7763),
            "ragged": (1_000_000, 64, 400_000), "mosi": (1_000_000, 20, 3016)}[kind]
    A, Vd = (76, 48) if kind == "mosi" else (300, 300)
    scaling = args.scaling or ("weak" if args.utts_per_gpu else "strong")
    T = args.tokens or dflt[1]
    V = args.vocab or dflt[2]
    D = 300
    if scaling == "strong":
        U_total = args.utts or args.utts_per_gpu or dflt[0]
        row0, U = Dist.shard_range(U_total, world, rank)
    else:
        U = args.utts_per_gpu or args.utts or dflt[0]
        U_total, row0 = U * world, U * rank
    if kind == "synthetic":
        inp = synth.device_shard(row0, U, T, V, D=D, A=300, Vd=300, seed=1000, device=dev)
    elif kind == "mosi":  # mosi_mmb2_config's inputs
        inp = synth.device_workload(U, T, V, D=D, A=A, Vd=Vd, seed=4000 + rank, device=dev)
    else:  # N = 1 configs (their own generators: ragged lengths, POM transcripts)
        inp = synth.device_workload(U, T, V, D=D, A=300, Vd=300, seed=1000 + rank, device=dev,
                                    mean_len=370.0 if kind == "pom" else None,
                                    poisson_len=40.0 if kind == "ragged" else None)
        inp.pop("lengths", None)
    ids = inp["ids"]
    text_rows = None
    if kind in ("pom", "ragged"):
        text_rows = (ids != 0).sum().item() / U + (ids == 0).any(1).float().mean().item()
    torch.manual_seed(0)
    gen = models.AudioVisualGeneratorMultimodal(D, A, Vd, norm=None).to(dev)

    def allreduce(t):
        dist.all_reduce(t)

    assert U_total >= D  # sklearn's direct (non-transposed) randomized-SVD branch
    step = P.FusedStep(inp, gen.networks(), allreduce=allreduce if world > 1 else None,
                       n_total=U_total, row0=row0, chunks=args.chunks,
                       side_cus=args.side_cus, side_layout=args.side_layout)
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        step.run()
    torch.cuda.synchronize()

    # timed region: K steps, barrier + sync on both sides.  Then K more steps
    # with HIP events recorded on the stream each phase is launched on
    # (FusedStep.run trace) for phase_ms and the kernels' launch durations --
    # outside the timed region (r05: ~12 event markers per step had been
    # inside it)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step.run()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    step.check()  # ids in range, no all-zero-weight utterance, finite PC (every rank)
    traces = [dict() for _ in range(args.steps)]
    for k in range(args.steps):
        step.run(trace=traces[k])
    torch.cuda.synchronize()
    step.check()
    if args.dump_rows:
        dump_rows(args.dump_rows, rank, row0, step)

    phase_ms = phase_times(traces, args.steps)
    ms_per_step = elapsed * 1e3 / args.steps
    value = U_total * args.steps / elapsed
    if rank != 0:
        dist.destroy_process_group()
        return 0

    utts_per_launch = U // len(step.bounds) if len(step.bounds) > 1 else U
    kb, kname = dominant_kernel(step, T, D, text_rows=text_rows)
    roof = stream_roofline(phase_ms, traces, args.steps, kb, utts_per_launch, kname, kind, T)
    if kind == "mosi":
        table_resident_roofline(roof, kb, utts_per_launch, D, T, narrow_fused=step.narrow_fused)
    pb = path_bytes(T, D, A, Vd, text_rows=text_rows)
    mfma = mfma_rooflines(step, phase_ms, U, D)
    wl = {"synthetic": "configs[3]: synthetic utterances x 40 tokens/frames x 3 modalities x "
                       "300d, V = 400k, Zipf(1.1) ids, SIF(+PC removal) + closed-form MMB2",
          "pom": "configs[2]: POM-shaped (V=7763, w0=1.0, transcripts padded to 1357, ~370 "
                 "tokens, aligned frames) x 3 modalities x 300d, SIF(+PC removal) + MMB2",
          "ragged": "configs[3] ragged: Poisson(40) lengths in [1, 64], padded with id 0 / -10 "
                    "frames, 3 x 300d, V = 400k, SIF(+PC removal) + MMB2",
          "mosi": "configs[1] MOSI-shaped: T = 20, A = 76, Vd = 48, V = 3016, Zipf(1.1) ids, "
                  "SIF(+PC removal) + closed-form MMB2"}[kind]
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "utterance-embeds/s",
        "n_gpus": world,
        "ranks_seen": ranks_seen,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": DTYPE,
        "data": "synthetic (seeded, generated in HBM; no dataset or checkpoint)",
        "config": {"workload": wl, "utts_total": U_total, "utts_rank0": U, "tokens": T,
                   "vocab": V, "dims": [D, A, Vd],
                   "parallelism": f"dp{world} (contiguous utterance shards of one split, "
                                  f"{scaling} scaling) + one all-reduce of the 300x300 fp64 Gram "
                                  f"({'RCCL' if args.dist_backend == 'nccl' else 'gloo'})"
                                  + (", all ranks on GPU 0" if args.share_device else "")},
        "roofline": roof,
        "path_roofline": {"bytes_per_utt": round(pb, 1),
                          "achieved": round(pb * U / (ms_per_step / 1e3) / 1e9, 1),
                          "unit": "GB/s per GPU", "peak": HBM_PEAK_GBS,
                          "frac": round(pb * U / (ms_per_step / 1e3) / 1e9 / HBM_PEAK_GBS, 4)},
        "phase_ms": {k: round(v, 4) for k, v in phase_ms.items()},
        "mfma_rooflines": mfma,
        "chunks": len(step.bounds),
    }
    if "pc_remove" in phase_ms:  # separate removal pass: x read, SIF row written
        rb = 2 * 4 * D
        ach = rb * U / (phase_ms["pc_remove"] / 1e3) / 1e9
        out["pc_remove_roofline"] = {"bound": "hbm", "achieved": round(ach, 1),
                                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                     "frac": round(ach / HBM_PEAK_GBS, 4), "bytes_per_utt": rb,
                                     "ms": round(phase_ms["pc_remove"], 4)}
    if world > 1:
        out["phase_ms"].setdefault("allreduce", None)
    if args.dump_rows:
        out["dump_rows"] = args.dump_rows
    cpu = None
    extras = world == 1 and not args.only_main and kind == "synthetic"
    if extras:
        sizes = [u for u in (500_000, 250_000, 125_000) if u < U]
        prs = per_rank_steps(P, inp, gen, args.steps, args.warmup, sizes)
        prs[str(U)] = {"utts": U, "ms_per_step": round(ms_per_step, 4), "value": round(value, 1),
                       "phase_ms": out["phase_ms"]}
        out["per_rank_steps"] = prs
        out["aux_warmup_min_s"] = AUX_WARMUP_S  # per_rank_steps / configs_measured warmup floor
        proj = {}
        for n_r in (2, 4, 8):
            key = str(U // n_r)
            if key in prs:
                proj[str(n_r)] = round(ms_per_step / prs[key]["ms_per_step"], 3)
        out["strong_scaling_projection"] = {
            "speedup": proj, "note": "t(1M) / t(1M / N) on one GPU: the per-rank step of the "
                                     "N-GPU strong-scaling run without the Gram all-reduce "
                                     "and the rank skew"}
        if step.stream_project:
            out["step_two_kernels"] = two_kernel_step(P, step, gen)
        out["projection_fp32_mfma"] = time_fp32_projection(P, step)
        out["stream_uniform_ids"] = stream_uniform_ids(P, step, kb)
    sample = None
    if not args.no_cpu_baseline and world == 1:
        n_cpu = args.cpu_sample if T <= 64 else max(1, args.cpu_sample * 40 // T)
        sample = host_sample(inp, n_cpu)
    gen_cpu = models.AudioVisualGeneratorMultimodal(D, A, Vd, norm=None)
    gen_cpu.load_state_dict({k: v.cpu() for k, v in gen.state_dict().items()})
    del step, inp, ids
    torch.cuda.empty_cache()
    if extras:
        cm = {}
        for name, fn in (("mmb1_sif_mosi", lambda: mmb1_sif_mosi_config(dev)),
                         ("mosi_mmb2", lambda: mosi_mmb2_config(P, models, synth, dev, 5, 2)),
                         ("dataset_splits", lambda: dataset_splits_config(P, models, synth, dev)),
                         ("ragged", lambda: ragged_config(P, models, synth, dev, 5, 2, U)),
                         ("pom", lambda: pom_config(P, models, synth, dev, 5, 2)),
                         ("regressor", lambda: regressor_config(dev)),
                         ("latent_step", lambda: latent_step_config(dev))):
            try:
                cm[name] = fn()
            except Exception as exc:  # keep the headline line even if an extra leg fails
                log(f"configs_measured.{name} failed: {exc!r}")
                cm[name] = {"error": repr(exc)}
            torch.cuda.empty_cache()
        out["configs_measured"] = cm
    if sample is not None:
        try:
            cpu = cpu_baseline(sample, gen_cpu, sample[2].shape[0])
        except Exception as exc:  # keep the GPU line even if the host leg fails
            log(f"cpu baseline failed: {exc!r}")
    out["cpu_baseline"] = cpu
    try:
        ceil = hbm_ceilings(dev)
        out["hbm_ceilings"] = {"copy_gbs": ceil["copy"], "read_gbs": ceil["read"],
                               "copy_config": ceil["copy_config"],
                               "read_config": ceil["read_config"], "sweep": ceil["sweep"],
                               "note": "libmmb float4 probes (mmb_probe_copy / mmb_probe_read) "
                                       "over 4 GiB in this process, best of the sweep; copy "
                                       "counts read + write"}
        annotate_ceilings(out, ceil)
    except Exception as exc:  # keep the line
        log(f"hbm ceilings failed: {exc!r}")
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
