#!/usr/bin/env python3
"""PCIe-inclusive rate of the numpy boundary.

sif.get_sentence_embeddings (sif.py:84-94) takes host numpy arrays and returns
a float64 numpy array, so a call pays the uploads (word table, weights,
int64 ids) and the f64 download on top of the device work.  Timed here
end to end (wall clock, synchronised) against the same a1-a5 work on
device-resident inputs (pipeline.sif_embeddings, f64 output on device), at
the POM shape (configs[2]: V = 7763, 303 transcripts padded to 1357) and the
bench shape (configs[3] text side: V = 400k, 1M utterances x 40 tokens).

    python tools/host_boundary_bench.py [--reps 5]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-baselines_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def wall(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import pipeline as P
    import sif
    import synth

    dev = torch.device("cuda", 0)
    out = {"what": "sif.get_sentence_embeddings (numpy in, f64 numpy out) vs device-resident a1-a5",
           "cases": []}
    for name, N, L, V, mean_len in (("configs[2] POM shape", 303, 1357, 7763, 370.0),
                                    ("configs[3] bench shape (text side)", 1_000_000, 40, 400_000, None)):
        E = synth.word_table(V, 300, seed=1)
        wt = synth.sif_weights(V, w0=1.0)
        ids = synth.token_ids(N, L, V, seed=2, ragged=mean_len is not None)
        ids64 = ids.astype(np.int64)
        host_ms = wall(lambda: sif.get_sentence_embeddings(E, wt, ids64), args.reps)
        table = torch.tensor(E, device=dev)
        w32 = torch.tensor(wt, device=dev, dtype=torch.float32)
        ids_d = torch.as_tensor(ids64, device=dev)
        dev_ms = wall(lambda: P.sif_embeddings(table, ids_d, wtab32=w32, npc=1,
                                               out_dtype=torch.float64), args.reps)
        host_bytes = E.nbytes // 1 + wt.nbytes + ids64.nbytes + N * 300 * 8
        out["cases"].append({"case": name, "N": N, "L": L, "V": V,
                             "host_boundary_ms": round(host_ms, 3),
                             "device_resident_ms": round(dev_ms, 3),
                             "host_boundary_utt_per_s": round(N / host_ms * 1e3, 1),
                             "device_resident_utt_per_s": round(N / dev_ms * 1e3, 1),
                             "pcie_bytes": host_bytes})
        del table, w32, ids_d
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
