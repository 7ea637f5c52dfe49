#!/usr/bin/env python3
"""MMB2 rounding against the reference's own fp32 rounding (g4 fixtures).

For each g4 case prints max row-relative error vs the reference's f64 rows
(cs_f64) of: the reference's fp32 run (cs_f32), the gpu2 drop-in (mm2_stream
+ fp16x3 projection), the fused stream + projection kernel (FusedStep), the
fp32-MFMA projection.  Also the per-row ratio statistics.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import pipeline as P  # noqa: E402
from oracle import mmb2_oracle as M  # noqa: E402
from test_gpu_mmb2 import _drop_in_call, _inputs  # noqa: E402


def rows_err(y, ref):
    return np.abs(y - ref).max(1) / np.abs(ref).max(1)


def main():
    dev = torch.device("cuda", 0)
    for case in ("g4_mmb2_mosi", "g4_mmb2_syn"):
        z = np.load(os.path.join(ROOT, "tests", "golden", case + ".npz"))
        gen, E, ids, audio, visual, weights = _inputs(z, dev)
        ref64 = z["cs_f64"]
        e_ref = rows_err(z["cs_f32"].astype(np.float64), ref64)
        drop = _drop_in_call(gen, E, ids, audio, visual, weights, dev).cpu().numpy()
        n, t = ids.shape
        inputs = {"table": torch.tensor(E, device=dev),
                  "wtab": torch.tensor(weights, device=dev, dtype=torch.float32),
                  "ids": torch.as_tensor(ids, dtype=torch.int32, device=dev),
                  "audio": torch.tensor(audio, device=dev), "visual": torch.tensor(visual, device=dev)}
        step = P.FusedStep(inputs, gen.to(dev).networks())
        _, fused = step.run()
        fused = fused.cpu().numpy()
        A, Vd = audio.shape[-1], visual.shape[-1]
        num, s32, aux = P.mm2_stream(n, t, 300, A, Vd, inputs["audio"], inputs["visual"],
                                     ids32=inputs["ids"], table=inputs["table"],
                                     wtab32=inputs["wtab"], s_half=False)
        p32 = P.mm2_project(s32, num, aux, step.proj).cpu().numpy()
        for name, y in (("ref_fp32", z["cs_f32"]), ("dropin_x3", drop), ("fused", fused),
                        ("fp32_mfma", p32)):
            e = rows_err(y.astype(np.float64), ref64)
            print(f"{case:14s} {name:10s} max {e.max():.3e} median {np.median(e):.3e} "
                  f"ratio-to-ref max {np.max(e / np.maximum(e_ref, 1e-300)):.2f}")


if __name__ == "__main__":
    main()
