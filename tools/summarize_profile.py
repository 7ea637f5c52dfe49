#!/usr/bin/env python3
"""Summarise a tools/gpu_profile.sh session into profiles/<tag>_*.

* kernel stats (rocprofv3 --kernel-trace --stats) with short names;
* HBM traffic per launch of each libmmb kernel from the two PMC passes:
  FETCH_SIZE and WRITE_SIZE are KB; on gfx950 FETCH_SIZE counts exactly half
  the bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM), so
      hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
  (an upper estimate for narrower accesses, which that section leaves
  uncalibrated);
* the bench JSON line of the session.

Usage: python tools/summarize_profile.py gpurun_out/r01 r01
"""
import csv
import json
import os
import re
import subprocess
import sys


def demangle(name):
    if name.startswith("_Z"):
        try:
            out = subprocess.run(["c++filt", name], capture_output=True, text=True,
                                 check=True).stdout.strip()
            if out != name:
                return out
        except (OSError, subprocess.CalledProcessError):
            pass
    if name.startswith("_ZN"):  # binutils c++filt lacks _Float16 (DF16_): keep the nested name
        parts, i = [], 3
        while i < len(name) and name[i].isdigit():
            j = i
            while name[j].isdigit():
                j += 1
            n = int(name[i:j])
            parts.append(name[j:j + n])
            i = j + n
        if parts:
            return "::".join(parts)
    return name


def short(name):
    name = re.sub(r"\(.*", "", demangle(name))
    name = name.replace("void ", "").replace("mmb::", "")
    return name[:70]


def main(src, tag):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(root, "profiles")
    os.makedirs(prof, exist_ok=True)
    lines = [f"# rocprofv3 summary — {tag}", ""]
    bench = json.load(open(os.path.join(src, "bench.json")))
    lines += ["## bench line", "", "```json", json.dumps(bench, indent=1), "```", ""]
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    # the traced process's own bench line: its HIP-event stream-kernel average
    # against rocprofv3's average for the same launches (same process; the
    # untraced bench above is another process, and the stream kernel varies
    # a few % from process to process on one box)
    tb_path = os.path.join(src, "trace_bench.json")
    if os.path.exists(tb_path):
        tb = json.load(open(tb_path))
        ev = tb["roofline"]["avg_launch_ms"]
        rp = [float(r["AverageNs"]) / 1e6 for r in stats if "utt_wave_kernel" in r["Name"]
              or "utt_stream_kernel" in r["Name"]]
        lines += ["## traced run: HIP events vs rocprofv3 (same process)", "",
                  f"stream kernel avg launch: HIP events {ev:.4f} ms, rocprofv3 "
                  f"{rp[0] if rp else float('nan'):.4f} ms; traced-run value {tb['value']:.1f} utt/s, "
                  f"{tb['ms_per_step']:.4f} ms/step", ""]
    lines += ["## kernel stats (`rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 10 "
              "--warmup 3 --no-cpu-baseline`)", "",
              "| kernel | calls | avg ms | total % |", "|---|---|---|---|"]
    for r in stats:
        lines.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e6:.4f} | "
                     f"{float(r['Percentage']):.2f} |")
    lines.append("")

    def pmc(path):
        out = {}
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            if "mmb" not in demangle(r["Kernel_Name"]):
                continue
            out.setdefault(k, []).append(float(r["Counter_Value"]))
        return out

    fetch = pmc(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    write = pmc(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    lines += ["## HBM traffic per launch (PMC; `(2*FETCH_SIZE + WRITE_SIZE) * 1024`)", "",
              "| kernel | launches | FETCH_SIZE KB | WRITE_SIZE KB | HBM bytes/launch |",
              "|---|---|---|---|---|"]
    traffic = {}
    for k in sorted(fetch):
        f = sum(fetch[k]) / len(fetch[k])
        w = sum(write.get(k, [0.0])) / max(1, len(write.get(k, [0.0])))
        b = (2 * f + w) * 1024
        traffic[k] = b
        lines.append(f"| `{k}` | {len(fetch[k])} | {f:.0f} | {w:.0f} | {b:.4g} |")
    lines.append("")
    stream = [v for k, v in traffic.items() if "utt_stream_kernel" in k or "utt_wave_kernel" in k]
    cfg = bench["config"]
    tj = {"tag": tag, "utts_per_launch": cfg["utts_per_gpu"], "tokens": cfg["tokens"],
          "mm2_stream_hbm_bytes_per_launch": stream[0] if stream else None,
          "per_kernel_hbm_bytes_per_launch": traffic}
    with open(os.path.join(prof, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(lines))
    with open(os.path.join(prof, f"{tag}_traffic.json"), "w") as f:
        json.dump(tj, f, indent=1)
    with open(os.path.join(prof, "traffic_latest.json"), "w") as f:
        json.dump(tj, f, indent=1)
    with open(os.path.join(prof, f"{tag}_kernel_stats.csv"), "w") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "avg_ns", "total_ns", "percent"])
        for r in stats:
            w.writerow([short(r["Name"]), r["Calls"], r["AverageNs"], r["TotalDurationNs"], r["Percentage"]])
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
