"""CPU: bench.py's contract pieces that need no GPU.

* `bench.py --gpus 2` outside torchrun starts the ranks itself (a child
  torch.distributed.run), here in --launch-check mode: both ranks join a gloo
  group and all-reduce a one, rank 0 reports what it saw.
* the algorithmic byte counts the roofline divides by.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 3])
def test_bench_self_launches_n_ranks(n):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                        "--launch-check"], capture_output=True, text=True, timeout=300, env=env,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["ranks_seen"] == n and out["allreduce_sum"] == n
    assert out["pid"] != os.getpid()
    assert "launching %d ranks" % n in r.stderr


def test_single_rank_launch_check_runs_in_process():
    env = {k: v for k, v in os.environ.items() if k != "WORLD_SIZE"}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--launch-check"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["ranks_seen"] == 1
    assert "launching" not in r.stderr


def test_algorithmic_bytes_match_survey():
    sys.path.insert(0, ROOT)
    import bench

    assert bench.path_bytes(40, 300, 300, 300) == 149_120  # SURVEY §8d B_utt at configs[3]
    assert bench.stream_kernel_bytes(40, 300, 300, 300) == 152_728
    # ragged: id-0 pad rows counted once per utterance (text_rows = n_tok + 1)
    assert bench.path_bytes(64, 300, 300, 300, text_rows=41) == 8 * 64 + 1200 * 41 + 2400 * 64 + 4800
