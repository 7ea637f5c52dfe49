"""Cross-checks of the measured kernel variants against the product defaults.

The product library (libmmb.so) carries only the default kernels and reads
no environment variable.  The variants the design notes measured -- the
projection's 32x32x16 / un-pipelined / register-A (3) / 256-row (4) /
register-B (6) kernels and its tile-layout epilogue, the stream kernel's
load/store policies and grid sizes, the fused kernel's group-at-a-time and
pipelined streamers and its unbalanced tail, the narrow fused kernel's
4-wave teams, the int8 Gram with x staged in LDS, the one-row PC removal -- live in
the tools build, libmmb_diag.so (`make diag`: tools/diag/, plugged into the
product sources' MMB_HOOK_* points), where MMB_* knobs
select them per launch.  This script runs in a child process that loads
that build explicitly (mmb_lib.load(path), tests/test_gpu_variants.py) and asserts
that each variant reproduces the default path: bit-identical where the
variant sums in the same order, within the stated bar otherwise.

    make -C multimodal-baselines_amd/csrc diag && python tests/variant_checks.py <group>
"""
from __future__ import annotations

import contextlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-baselines_amd")]
DIAG_LIB = os.path.join(ROOT, "tools", "diag", "libmmb_diag.so")

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mmb_lib as L  # noqa: E402
import models  # noqa: E402
import pipeline as P  # noqa: E402
import synth  # noqa: E402
from oracle import mmb2_oracle as M  # noqa: E402

TOL = 1e-5


@contextlib.contextmanager
def knobs(**kv):
    """Set MMB_* knobs of the tools build for the launches inside the block."""
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update({k: str(v) for k, v in kv.items()})
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _gen(dev, A=300, Vd=300):
    torch.manual_seed(0)
    return models.AudioVisualGeneratorMultimodal(300, A, Vd, norm=None).to(dev)


def check_projection(dev):
    """Projection variants 3 (A fragments straight from HBM into registers),
    4 (256-row tiles) and 6 (B straight from L2 into registers) sum every
    16x16 tile in the default kernel's MFMA order and share its epilogue:
    MMB2 and PC-removed rows bit-identical, ragged last tiles included.  The
    32x32x16 kernel (0), the un-pipelined 16x16x32 kernel (1) and the
    tile-layout epilogue agree to the removal's dot order / the 1e-5 bar."""
    for N in (700, 128, 129, 1000):
        inp = synth.device_workload(N, 40, 5000, A=300, Vd=300, seed=41, device=dev)
        step = P.FusedStep(inp, _gen(dev).networks(), stream_project=False)
        s1, m1 = [t.clone() for t in step.run()]
        for variant in ("3", "4", "6"):
            with knobs(MMB_PROJ_VARIANT=variant):
                step.sif.zero_()
                step.mmb2.zero_()
                s3, m3 = step.run()
                torch.cuda.synchronize()
            assert torch.equal(m1, m3), ("mmb2", N, variant)
            assert torch.equal(s1, s3), ("sif", N, variant)
        for kv in ({"MMB_PROJ_VARIANT": "0", "MMB_STREAM_POLICY": "0"}, {"MMB_PROJ_VARIANT": "1"},
                   {"MMB_STREAM_POLICY": "7", "MMB_STREAM_GRID_MULT": "8"},
                   {"MMB_STREAM_POLICY": "13"}, {"MMB_PROJ_ROWEPI": "0"}):
            with knobs(**kv):
                s2, m2 = [t.clone() for t in step.run()]
                torch.cuda.synchronize()
            # the 32x32x16 kernel's tail reduces the removal's f64 dot with
            # shuffles, not DPP: the SIF rows agree to that order
            assert M.row_rel_err(s2.cpu().numpy(), s1.cpu().numpy()) < 1e-6, (N, kv)
            assert M.row_rel_err(m2.cpu().numpy(), m1.cpu().numpy()) < TOL, (N, kv)
    print("projection: variants 0/1/3/4/6, tile epilogue, stream policies 0/7/13 ok")


# (N, T, A, Vd, dense text, bad ids)
FUSED_CASES = [(2048, 40, 300, 300, False, False), (15, 40, 300, 300, False, False),
               (700, 64, 300, 300, False, True), (999, 33, 260, 292, False, False),
               (97, 40, 300, 20, False, False), (300, 17, 300, 256, False, False),
               (5003, 24, 300, 300, False, True), (50, 16, 300, 300, False, False),
               (500, 40, 300, 300, True, False), (49, 40, 100, 300, False, False),
               (30011, 40, 300, 300, False, False)]


def fused_case(dev, N, T, A, Vd, bad):
    """Seeded inputs and the merged projection of one FUSED_CASES entry."""
    inp = synth.device_workload(N, T, 20_000, A=A, Vd=Vd, seed=71, device=dev)
    if bad:  # negative ids wrap; ids >= V are flagged and contribute zero rows
        inp["ids"][3, 5] = -7
        inp["ids"][N // 2, T - 1] = 20_000 + 11
        inp["ids"][N - 1, 0] = -20_001
    proj = P.MMB2Projection(_gen(dev, A, Vd).networks(), 300, A, Vd, T, dev)
    return inp, proj


def fused_outputs(inp, proj, n, t, a, vd, dense=False):
    """One mmb_mm2_stream_project launch (whatever the loaded library's
    default streamer is); every output cloned."""
    d = 300
    flag = torch.zeros(1, dtype=torch.int32, device=inp["audio"].device)
    colmax = torch.empty(d, dtype=torch.int32, device=flag.device)
    ws = torch.empty(L.query("mmb_mm2_colmax_ws_bytes", d), dtype=torch.uint8, device=flag.device)
    kw = dict(ids32=inp["ids"], table=inp["table"], wtab32=inp["wtab"])
    if dense:
        ids = inp["ids"].long()
        kw = dict(text_dense=inp["table"][ids.clamp(min=0)].contiguous(),
                  w_dense=inp["wtab"][ids.clamp(min=0)] * (ids >= 0))
    x, aux, m = P.mm2_stream_project(n, t, d, a, vd, inp["audio"], inp["visual"], proj,
                                     flag=flag, colmax=colmax, colmax_ws=ws, **kw)
    torch.cuda.synchronize()
    return [v.clone() for v in (x, aux, m, colmax, flag)]


def _fused_outputs(inp, proj, n, t, a, vd, pipe, dense=False, balanced=False):
    with knobs(MMB_FUSED_PIPE=int(pipe), MMB_FUSED_BALANCED=1 if balanced else 0):
        return fused_outputs(inp, proj, n, t, a, vd, dense=dense)


def check_fused_streamer(dev):
    """The pipelined streamers of utt_fused_kernel (MMB_FUSED_PIPE=1: two
    frame groups in flight across group, row and text-token boundaries; =2,
    the product default: also across piece and batch boundaries) against the
    group-at-a-time streamer: x, aux, MMB2 rows, column bounds and the flag
    word bit-identical -- partial batches, partial last groups (T = 33, 17),
    the 3-group minimum (T = 24; T = 16 falls back), narrow frames, dense
    text, negative and out-of-range ids -- with and without the balanced tail
    (N = 30011: two full rounds of 256 x 48 rows and a 5,435-row tail)."""
    names = ["x", "aux", "mmb2", "colmax", "flag"]
    dump = os.environ.get("VARIANT_DUMP")
    for ci, (N, T, A, Vd, dense, bad) in enumerate(FUSED_CASES):
        inp, proj = fused_case(dev, N, T, A, Vd, bad)
        ref = _fused_outputs(inp, proj, N, T, A, Vd, pipe=False, dense=dense)
        if dump:  # the group-at-a-time streamer's outputs, for the product-library comparison
            np.savez(os.path.join(dump, f"fused_{ci}.npz"),
                     **{nm: r.cpu().numpy() for nm, r in zip(names, ref)})
        for pipe, bal in [(1, False), (1, True), (0, True), (2, True), (2, False)]:
            got = _fused_outputs(inp, proj, N, T, A, Vd, pipe=pipe, dense=dense, balanced=bal)
            for nm, r, g in zip(names, ref, got):
                assert torch.equal(torch.nan_to_num(r, nan=7.0), torch.nan_to_num(g, nan=7.0)), \
                    (nm, N, T, pipe, bal)
        assert (int(ref[4].item()) != 0) == bad
    print(f"fused streamer: {len(FUSED_CASES)} shapes x 5 streamer / tail variants bit-identical")


def check_fused_order(dev):
    """The fused kernel's dynamic batch order (from 16 rounds of batches on:
    streamers draw 48-row batches from a per-launch counter, the last round
    in 12-row units) against the static round robin (MMB_FUSED_DYN=0): x,
    aux, MMB2 rows, column bounds and the flag bit-identical -- N = 200,018
    rows (4,168 batches >= 16 x 256) leaves a last unit of 2 rows, so two
    streamer waves see a unit without rows of their own and only pad its
    fill counts; the same launch twice (the counter re-zeroed per launch)."""
    names = ["x", "aux", "mmb2", "colmax", "flag"]
    N, T, A, Vd = 200_018, 24, 64, 64
    assert (N + 47) // 48 >= 16 * min(256, L.cu_count(dev)), "too few rows for the dynamic order"
    inp, proj = fused_case(dev, N, T, A, Vd, False)
    with knobs(MMB_FUSED_DYN=0):
        ref = fused_outputs(inp, proj, N, T, A, Vd)
    for rep in range(2):
        with knobs(MMB_FUSED_DYN=1):
            got = fused_outputs(inp, proj, N, T, A, Vd)
        for nm, r, g in zip(names, ref, got):
            assert torch.equal(torch.nan_to_num(r, nan=7.0), torch.nan_to_num(g, nan=7.0)), (nm, rep)
    assert int(ref[4].item()) == 0
    print("fused order: dynamic batch order bit-identical to the round robin (2 launches)")


def check_remove_rows(dev):
    """pc_remove1_kernel (one PC, R = 2 / 4 / 8 rows per wave in flight, the
    PC in registers) against pc_remove_kernel (MMB_PC_REMOVE_R=0):
    bit-identical rows -- row counts not multiples of R, narrow rows, a count
    divisor -- and within 1e-6 of the f64 removal."""
    for n, d, with_cnt in [(1, 300, False), (5, 300, True), (1003, 300, False),
                           (4099, 300, True), (777, 260, False), (130, 292, True)]:
        g = torch.Generator(device=dev).manual_seed(5)
        x = torch.randn(n, d, generator=g, device=dev) * 3 + 0.5
        cnt = torch.randint(1, 40, (n,), generator=g, device=dev).float() if with_cnt else None
        pc = torch.randn(1, d, generator=g, device=dev, dtype=torch.float64)
        pc /= torch.linalg.norm(pc)
        outs = []
        for r in ("0", "4", "2", "8"):
            with knobs(MMB_PC_REMOVE_R=r):
                outs.append(P.remove_pc(x, cnt, pc).clone())
                torch.cuda.synchronize()
        for o in outs[1:]:
            assert torch.equal(o, outs[0]), (n, d)
        xs = x.double() / (cnt.double()[:, None] if with_cnt else 1.0)
        ref = xs - (xs @ pc.T) @ pc
        assert (outs[0].double() - ref).abs().max().item() <= 1e-6 * xs.abs().max().item()
    print("remove rows: R = 0/2/4/8 bit-identical")


def check_gram_schedules(dev):
    """The int8 Gram's timing-only ablations are wrong by design; its product
    schedule (MMB_GRAM_DIAG unset) must equal the product library's Gram --
    checked here against the exact f64 Gram to the int8 format's 2e-9 -- and
    the kernel with x staged in LDS by DMA (MMB_GRAM_I8_SHAPE=6,
    gram_i8s_kernel: the same digits and exact level sums) equals it bit for
    bit, a partial last chunk included (77,777 rows)."""
    for n in (5000, 77_777):
        g = torch.Generator(device=dev).manual_seed(n)
        x = torch.randn(n, 300, generator=g, device=dev) * 0.3
        cm = P.colmax(x)
        G8 = P.gram_i8(x, cm).clone()
        with knobs(MMB_GRAM_I8_SHAPE=6):
            Gs = P.gram_i8(x, cm).clone()
        G64 = P.gram(x, None)
        torch.cuda.synchronize()
        assert (G8 - G64).abs().max().item() <= 2e-9 * G64.abs().max().item(), n
        assert torch.equal(G8, Gs), n
    print("gram: int8 schedule within 2e-9 of f64; the LDS-staged kernel bit-identical")


def check_narrow_teams(dev):
    """The narrow fused kernel (MOSI widths) run as two 4-wave teams with their
    own 16-row batches, LDS halves and barriers (MMB_NF_TEAMS=1, and =2 with
    team 1 a stream phase late) against the product's 32-row workgroup
    batches: every row is computed the same way whichever team takes it, so
    x, aux, the MMB2 and SIF rows, the column bounds and the PC are
    bit-identical -- 1, 2 and 4 utterances per wave (N = 1284, 6000, 40,000)."""
    for n in (1284, 6000, 40_000):
        inp = synth.device_workload(n, 20, 3016, A=76, Vd=48, seed=70 + n % 97, device=dev)
        st = P.FusedStep(inp, _gen(dev, 76, 48).networks(), narrow_fused=True)
        assert st.narrow_fused
        outs = {}
        for v in ("0", "1", "2"):
            with knobs(MMB_NF_TEAMS=v):
                st.run(check=True)
                torch.cuda.synchronize()
            # (colmax: None below the int8 Gram's row threshold)
            outs[v] = [None if t is None else t.clone()
                       for t in (st.x, st.aux, st.mmb2, st.sif, st.colmax, st.pc)]
        for v in ("1", "2"):
            for a, b in zip(outs["0"], outs[v]):
                assert (a is None and b is None) or torch.equal(a, b), (n, v)
    print("narrow teams: two 4-wave teams bit-identical to the workgroup batches")


def check_timeouts(dev):
    """The bounded hand-over waits' timeout path: the fused stream +
    projection kernel with its wait budget cut to one poll
    (mmb_diag_fused_wait_iters), the multi-workgroup PC solve with
    workgroup 1 never arriving (mmb_diag_pc_skip_arrival) -- the count its
    waits poll for cannot be reached whatever the arrival skew, so the
    timeout is deterministic (r05: a one-poll budget alone raced the
    co-resident workgroups' arrivals and passed on the driver's box).  Both
    end (no hang), report MMB_FLAG_SYNC_TIMEOUT, leave a NaN PC, and the
    callers raise RuntimeError; with the product behaviour restored the same
    step and solve reproduce their results bit for bit."""
    lib = L.load()
    inp = synth.device_workload(20_000, 40, 20_000, seed=81, device=dev)
    step = P.FusedStep(inp, _gen(dev).networks(), stream_project=True)
    assert step.stream_project
    s0, m0 = [t.clone() for t in step.run(check=True)]
    try:
        assert lib.mmb_diag_fused_wait_iters(1) == 0
        step.run()
        torch.cuda.synchronize()
        assert int(step.flag.item()) & L.MMB_FLAG_SYNC_TIMEOUT
        try:
            step.check()
        except RuntimeError as e:
            assert "timed out" in str(e)
        else:
            raise AssertionError("FusedStep.check did not raise on the hand-over timeout")
    finally:
        assert lib.mmb_diag_fused_wait_iters(1 << 23) == 0
    step.reset()
    s1, m1 = step.run(check=True)
    assert torch.equal(s0, s1) and torch.equal(m0, m1)

    G = step.G.clone()
    z0 = torch.randn((300, 11), dtype=torch.float64, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    pc0 = P.pc_solve(G, z0, 1, False, flag=flag).clone()
    torch.cuda.synchronize()
    assert int(flag.item()) == 0
    try:
        assert lib.mmb_diag_pc_wait_iters(256) == 0
        assert lib.mmb_diag_pc_skip_arrival(1) == 0
        pcx = P.pc_solve(G, z0, 1, False, flag=flag)
        torch.cuda.synchronize()
        assert int(flag.item()) & L.MMB_FLAG_SYNC_TIMEOUT
        assert bool(torch.isnan(pcx).all())  # never a stale PC
        # callers that pass no flag raise too (pc_solve's own flag), and so
        # does the composed a1-a5 path
        for call in (lambda: P.pc_solve(G, z0, 1, False),
                     lambda: P.sif_embeddings(inp["table"], inp["ids"][:2000], wtab32=inp["wtab"])):
            try:
                call()
            except RuntimeError as e:
                assert "timed out" in str(e)
            else:
                raise AssertionError("a no-flag PC solve did not raise on the hand-over timeout")
    finally:
        assert lib.mmb_diag_pc_skip_arrival(-1) == 0
        assert lib.mmb_diag_pc_wait_iters(1 << 20) == 0
    flag.zero_()
    P.solve_workspace(300, dev)[:16].zero_()  # an aborted solve leaves its control words set
    pc1 = P.pc_solve(G, z0, 1, False, flag=flag)
    torch.cuda.synchronize()
    assert int(flag.item()) == 0 and torch.equal(pc0, pc1)
    print("timeouts: fused kernel and PC solve end, flag the timeout, recover bit for bit")


GROUPS = {"projection": check_projection, "fused_streamer": check_fused_streamer,
          "fused_order": check_fused_order,
          "remove_rows": check_remove_rows, "gram": check_gram_schedules,
          "narrow_teams": check_narrow_teams, "timeouts": check_timeouts}


def main(argv):
    want = argv[1:] or list(GROUPS)
    if not os.path.exists(DIAG_LIB):
        print(f"variant_checks: needs the tools build at {DIAG_LIB} (`make -C "
              f"multimodal-baselines_amd/csrc diag`)", file=sys.stderr)
        return 2
    L.load(DIAG_LIB)
    L.require_gpu()
    dev = torch.device("cuda", 0)
    for g in want:
        GROUPS[g](dev)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
