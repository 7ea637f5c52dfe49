#!/usr/bin/env python3
"""Summarise a tools/gpu_profile_r03.sh session (parts a and b) into profiles/<tag>_*:

* the bench line (headline + configs_measured);
* rocprofv3 kernel stats of the headline bench, and the traced process's own
  HIP-event stream-kernel average beside rocprofv3's;
* the same at the 125k-utterance per-rank size of the 8-GPU strong-scaling
  curve (bench.py --utts 125000);
* the e2e latent step's kernel stats (word_zsum_kernel etc.) and its bench
  line -> profiles/<tag>_latent_bench.json;
* per workload (synthetic / ragged / pom / mosi): HBM bytes per launch of every libmmb
  kernel from the FETCH_SIZE and WRITE_SIZE passes, hbm = (2 FETCH + WRITE) *
  1024 (gfx950: FETCH_SIZE counts half of wide coalesced reads,
  MI355X_MICROARCH.md §HBM), written to profiles/traffic[_<workload>]_latest.json
  for bench.py's roofline.traffic.

Usage: python tools/summarize_r03.py gpurun_out/r03s r03s
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_profile import demangle, short  # noqa: E402


def pmc(path):
    out = {}
    for r in csv.DictReader(open(path)):
        if "mmb" not in demangle(r["Kernel_Name"]):
            continue
        out.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
    return out


def main(src, tag):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    bench = json.load(open(os.path.join(src, "bench.json")))
    lines = [f"# rocprofv3 summary — {tag}", "", "## bench line (default invocation)", "", "```json",
             json.dumps(bench, indent=1), "```", ""]
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    tb = json.load(open(os.path.join(src, "trace_bench.json")))
    rp = [float(r["AverageNs"]) / 1e6 for r in stats
          if "utt_fused_kernel" in r["Name"] or "utt_wave_kernel" in r["Name"]]
    lines += ["## traced run: HIP events vs rocprofv3 (same process)", "",
              f"stream kernel avg launch: HIP events {tb['roofline']['avg_launch_ms']:.4f} ms, "
              f"rocprofv3 {rp[0] if rp else float('nan'):.4f} ms; traced-run value "
              f"{tb['value']:.1f} utt/s, {tb['ms_per_step']:.4f} ms/step", "",
              "## kernel stats (`rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 10 "
              "--warmup 3 --only-main --no-cpu-baseline`)", "",
              "| kernel | calls | avg ms | total % |", "|---|---|---|---|"]
    for r in stats:
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e6:.4f} | "
                     f"{float(r['Percentage']):.2f} |")
    lines.append("")
    with open(os.path.join(prof, f"{tag}_kernel_stats.csv"), "w") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "avg_ns", "total_ns", "percent"])
        for r in stats:
            w.writerow([short(r["Name"]), r["Calls"], r["AverageNs"], r["TotalDurationNs"],
                        r["Percentage"]])
    stats125 = list(csv.DictReader(open(os.path.join(src, "trace125k", "run_kernel_stats.csv"))))
    t125 = json.load(open(os.path.join(src, "trace125k_bench.json")))
    lines += ["## per-rank size of the 8-GPU strong-scaling curve (`bench.py --utts 125000 --steps 20 "
              "--warmup 3 --only-main --no-cpu-baseline` under rocprofv3)", "",
              f"step {t125['ms_per_step']:.4f} ms; phases (HIP events) {json.dumps(t125['phase_ms'])}", "",
              "| kernel | calls | avg ms | total % |", "|---|---|---|---|"]
    for r in stats125:
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e6:.4f} | "
                     f"{float(r['Percentage']):.2f} |")
    lines.append("")
    with open(os.path.join(prof, f"{tag}_kernel_stats_125k.csv"), "w") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "avg_ns", "total_ns", "percent"])
        for r in stats125:
            w.writerow([short(r["Name"]), r["Calls"], r["AverageNs"], r["TotalDurationNs"],
                        r["Percentage"]])
    lat_dir = os.path.join(src, "latent")
    if os.path.exists(lat_dir):
        lb = json.load(open(os.path.join(src, "latent_bench.json")))
        lst = list(csv.DictReader(open(os.path.join(lat_dir, "run_kernel_stats.csv"))))
        mmb = {short(r["Name"]): {"calls": int(r["Calls"]), "avg_us": round(float(r["AverageNs"]) / 1e3, 2),
                                  "percent": float(r["Percentage"])}
               for r in lst if "mmb" in demangle(r["Name"])}
        lb["rocprofv3_mmb_kernels"] = mmb
        lb["rocprofv3_note"] = ("rocprofv3 --kernel-trace --stats of tools/latent_bench.py --steps 30 "
                                "(the graph replays included); ms_per_step above is that traced "
                                "process's own timing")
        with open(os.path.join(prof, f"{tag}_latent_bench.json"), "w") as f:
            json.dump(lb, f, indent=1)
        lines += ["## e2e latent step (tools/latent_bench.py under rocprofv3)", "", "```json",
                  json.dumps(lb, indent=1), "```", ""]
    for wl in ("synthetic", "ragged", "pom", "mosi"):
        fetch = pmc(os.path.join(src, f"pmc_{wl}_FETCH_SIZE", "run_counter_collection.csv"))
        write = pmc(os.path.join(src, f"pmc_{wl}_WRITE_SIZE", "run_counter_collection.csv"))
        wb = json.load(open(os.path.join(src, f"pmc_{wl}_FETCH_SIZE.json")))
        lines += [f"## HBM traffic per launch — {wl} (PMC; `(2*FETCH_SIZE + WRITE_SIZE) * 1024`)",
                  "", f"workload: {wb['config']['workload']}; algorithmic stream-kernel bytes "
                  f"{wb['roofline']['algorithmic_bytes_per_utt']} per utterance", "",
                  "| kernel | launches | FETCH_SIZE KB | WRITE_SIZE KB | HBM bytes/launch |",
                  "|---|---|---|---|---|"]
        traffic = {}
        for k in sorted(fetch):
            fv = sum(fetch[k]) / len(fetch[k])
            wv = sum(write.get(k, [0.0])) / max(1, len(write.get(k, [0.0])))
            b = (2 * fv + wv) * 1024
            traffic[k] = b
            lines.append(f"| `{k}` | {len(fetch[k])} | {fv:.0f} | {wv:.0f} | {b:.4g} |")
        fused = [v for k, v in traffic.items() if "utt_fused_kernel" in k]
        stream = fused or [v for k, v in traffic.items()
                           if "utt_stream_kernel" in k or "utt_wave_kernel" in k
                           or "utt_narrow_kernel" in k]
        cfg = wb["config"]
        alg = wb["roofline"]["algorithmic_bytes_per_utt"] * cfg["utts_rank0"]
        if stream:
            lines += ["", f"stream kernel: {stream[0] / 1e9:.2f} GB measured vs {alg / 1e9:.2f} GB "
                          f"algorithmic per launch ({stream[0] / alg:.3f}x)"]
        lines.append("")
        tj = {"tag": tag, "workload": wl, "utts_per_launch": cfg["utts_rank0"],
              "tokens": cfg["tokens"], "mm2_stream_hbm_bytes_per_launch": stream[0] if stream else None,
              "phase": "mm2_stream_project" if fused else "mm2_stream",
              "algorithmic_bytes_per_launch": alg, "per_kernel_hbm_bytes_per_launch": traffic}
        name = "traffic_latest.json" if wl == "synthetic" else f"traffic_{wl}_latest.json"
        for fn in (f"{tag}_traffic_{wl}.json", name):
            with open(os.path.join(prof, fn), "w") as f:
                json.dump(tj, f, indent=1)
    with open(os.path.join(prof, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(lines))
    with open(os.path.join(prof, f"{tag}_bench.json"), "w") as f:
        json.dump(bench, f)
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
