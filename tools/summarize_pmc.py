#!/usr/bin/env python3
"""HBM bytes per launch of every libmmb kernel from a tools/gpu_pmc_r04.sh
session: hbm = (2 FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950: FETCH_SIZE counts
half of wide coalesced reads, MI355X_MICROARCH.md §HBM), written to
profiles/<tag>_traffic_<workload>.json and profiles/traffic[_<workload>]_latest.json
(bench.py's roofline.traffic for the step's dominant kernel), plus the step
total against the path's algorithmic bytes.

    python tools/summarize_pmc.py gpurun_out/r04p r04p mosi synthetic
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_profile import demangle, short  # noqa: E402

STREAM = (("utt_narrow_fused_kernel", "mm2_stream_project_narrow"),
          ("utt_fused_kernel", "mm2_stream_project"),
          ("utt_narrow_kernel", "mm2_stream"), ("utt_wave_kernel", "mm2_stream"),
          ("utt_stream_kernel", "mm2_stream"))


def pmc(path):
    out = {}
    for r in csv.DictReader(open(path)):
        if "mmb" not in demangle(r["Kernel_Name"]):
            continue
        out.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
    return out


def main(src, tag, workloads):
    prof = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
    lines = [f"# HBM traffic per launch — {tag} (PMC; `(2*FETCH_SIZE + WRITE_SIZE) * 1024`)", ""]
    for wl in workloads:
        fetch = pmc(os.path.join(src, f"pmc_{wl}_FETCH_SIZE", "run_counter_collection.csv"))
        write = pmc(os.path.join(src, f"pmc_{wl}_WRITE_SIZE", "run_counter_collection.csv"))
        wb = json.loads(open(os.path.join(src, f"pmc_{wl}_FETCH_SIZE.json")).read().strip().splitlines()[-1])
        cfg = wb["config"]
        traffic = {}
        lines += [f"## {wl}: {cfg['workload']}", "",
                  "| kernel | launches | FETCH_SIZE KB | WRITE_SIZE KB | HBM bytes/launch |",
                  "|---|---|---|---|---|"]
        for k in sorted(fetch):
            fv = sum(fetch[k]) / len(fetch[k])
            wv = sum(write.get(k, [0.0])) / max(1, len(write.get(k, [0.0])))
            traffic[k] = (2 * fv + wv) * 1024
            lines.append(f"| `{k}` | {len(fetch[k])} | {fv:.0f} | {wv:.0f} | {traffic[k]:.4g} |")
        stream, phase = None, None
        for key, ph in STREAM:
            hit = [v for k, v in traffic.items() if key in k]
            if hit:
                stream, phase = hit[0], ph
                break
        U = cfg["utts_rank0"]
        alg = wb["roofline"]["algorithmic_bytes_per_utt"] * U
        # per-step kernels: launched as often as the stream kernel (the bench's
        # HBM-ceiling probes and the one-off weight preparation excluded)
        nl = {k: len(v) for k, v in fetch.items()}
        skey = next((k for k in traffic if traffic[k] == stream), None)
        step_total = sum(v for k, v in traffic.items() if k and skey and nl[k] == nl[skey])
        path = wb["path_roofline"]["bytes_per_utt"] * U
        lines += ["", f"stream kernel ({phase}): {stream / 1e9:.3f} GB measured vs {alg / 1e9:.3f} GB "
                      f"algorithmic per launch ({stream / alg:.3f}x)" if stream else "no stream kernel",
                  f"every libmmb kernel of the step: {step_total / 1e9:.3f} GB"
                  + (f" vs the path's {path / 1e9:.3f} GB ({step_total / path:.3f}x)" if path else ""), ""]
        sha_f = os.path.join(src, "tree_sha.txt")  # tools/gpu_r05_final.sh: "tree: <sha>"
        sha = open(sha_f).read().split()[-1] if os.path.exists(sha_f) else None
        tj = {"tag": tag, "tree_sha": sha, "workload": wl, "utts_per_launch": U, "tokens": cfg["tokens"],
              "mm2_stream_hbm_bytes_per_launch": stream, "phase": phase,
              "algorithmic_bytes_per_launch": alg, "step_hbm_bytes": step_total,
              "path_bytes_per_step": path, "per_kernel_hbm_bytes_per_launch": traffic}
        name = "traffic_latest.json" if wl == "synthetic" else f"traffic_{wl}_latest.json"
        for fn in (f"{tag}_traffic_{wl}.json", name):
            with open(os.path.join(prof, fn), "w") as f:
                json.dump(tj, f, indent=1)
    with open(os.path.join(prof, f"{tag}_traffic.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
