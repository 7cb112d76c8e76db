"""The reduced-camera-system factorisation (csrc/cholesky.cpp) through
mi_ba_dense_cholesky, against the oracle's dense Cholesky and LAPACK.

Replaces the DENSE_SCHUR / SPARSE_SCHUR factorisation Ceres runs inside
BundleAdjuster::Solve (src/optim/bundle_adjustment.cc:276-306; Ceres 2.1 is
not vendored, so the oracle restates a plain column Cholesky).

Tolerances (f64):
  * look-ahead on vs off: bitwise identical L and info (same rocBLAS dgemm /
    dtrsm shapes in the same order; only the stream a panel runs on differs)
  * hand-written diagonal factor vs rocsolver_dpotrf, and vs the oracle /
    LAPACK: max|dL| <= 1e-12 * max|L| (different summation orders)
  * solve: max|dx| <= 1e-10 * max|x|
  * concurrent factorisations from two host threads: bitwise equal to the
    serial results (every call owns its stream, handles and workspace)
Sizes span several 512-wide panels with a ragged last panel and ragged
64-wide sub-panels (n = 1700 = 3 * 512 + 164, 2100).
"""
import threading

import numpy as np
import pytest
from scipy.linalg import solve_triangular

import mi_ba
import oracle

pytestmark = pytest.mark.gpu


def spd(n, seed=0):
    rng = np.random.default_rng(seed)
    G = rng.standard_normal((n, n // 2))
    return G @ G.T / n + np.diag(rng.uniform(0.5, 2.0, n))


@pytest.mark.parametrize("own", [2, 6])
@pytest.mark.parametrize("n", [1700, 2100])
def test_lookahead_bitwise_equal(gpu, n, own):
    A = spd(n, seed=n)
    L0, _, i0 = mi_ba.dense_cholesky(A, lookahead=0, own_diag=own)
    L1, _, i1 = mi_ba.dense_cholesky(A, lookahead=1, own_diag=own)
    assert i0 == 0 and i1 == 0
    assert np.array_equal(L0, L1)
    # repeatable
    L2, _, _ = mi_ba.dense_cholesky(A, lookahead=1, own_diag=own)
    assert np.array_equal(L1, L2)


@pytest.mark.parametrize("own", [2, 6, 0])
def test_factor_reads_lower_triangle_only(gpu, own):
    """The LM fills only S's column-major lower triangle (its row-major upper
    half, csrc/kernels.hip dense_u / schur_pairs): the strict upper
    triangle of A holds junk and must not be read."""
    n = 1300
    A = spd(n, seed=21)
    junk = np.triu(np.random.default_rng(5).uniform(-1e6, 1e6, (n, n)), 1)
    L, _, info = mi_ba.dense_cholesky(np.tril(A) + junk, own_diag=own)
    assert info == 0
    L_np = np.linalg.cholesky(A)
    assert np.abs(L - L_np).max() <= 1e-12 * np.abs(L_np).max()


@pytest.mark.parametrize("n", [64, 100, 512, 513, 1000])
def test_panel_kernel_small_and_ragged(gpu, n):
    """One-launch panel factor (own_diag 6) at one tile, a ragged tile, one
    full panel, one panel + 1 row, and a ragged last panel, against LAPACK."""
    A = spd(n, seed=n + 11)
    L, _, info = mi_ba.dense_cholesky(A, own_diag=6)
    assert info == 0
    L_np = np.linalg.cholesky(A)
    assert np.abs(L - L_np).max() <= 1e-12 * np.abs(L_np).max()


@pytest.mark.parametrize("n", [1700, 2100])
def test_factor_matches_oracle_and_lapack(gpu, n):
    A = spd(n, seed=7 + n)
    b = np.random.default_rng(n).standard_normal(n)
    L_o, info_o = oracle.cholesky(A)
    assert info_o == 0
    L_np = np.linalg.cholesky(A)
    x_ref = np.linalg.solve(A, b)
    scale = np.abs(L_o).max()
    for own in (6, 2, 1, 0):
        for panel in ((512, 256) if own == 6 else (512, 0)):
            L, x, info = mi_ba.dense_cholesky(A, b, panel=panel, own_diag=own)
            assert info == 0
            assert np.abs(L - L_o).max() <= 1e-12 * scale, (own, panel)
            assert np.abs(L - L_np).max() <= 1e-12 * scale, (own, panel)
            assert np.abs(x - x_ref).max() <= 1e-10 * np.abs(x_ref).max(), (own, panel)
    # the three triangular-solve variants on the default factor
    for solve in (0, 1, 2):
        L, x, info = mi_ba.dense_cholesky(A, b, solve=solve)
        assert info == 0
        assert np.abs(x - x_ref).max() <= 1e-10 * np.abs(x_ref).max(), solve


@pytest.mark.parametrize("n", [64, 65, 130, 12000])
def test_sync_free_solve_sizes(gpu, n):
    """Sync-free sweeps (one launch per direction) at one block, a ragged
    second block, and the C4 reduced-camera size (188 blocks, ragged last):
    against LAPACK on the same factor, and repeated solves (flag epochs) stay
    equal."""
    A = spd(n, seed=n + 3) if n <= 4096 else np.diag(np.linspace(1.0, 3.0, n)) + 1e-3
    b = np.random.default_rng(n).standard_normal(n)
    L, x, info = mi_ba.dense_cholesky(A, b, solve=2)
    assert info == 0
    y = solve_triangular(L, b, lower=True)
    x_ref = solve_triangular(L, y, lower=True, trans="T")
    assert np.abs(x - x_ref).max() <= 1e-10 * np.abs(x_ref).max()
    _, x1, _ = mi_ba.dense_cholesky(A, b, solve=1)
    assert np.abs(x - x1).max() <= 1e-12 * np.abs(x_ref).max()


@pytest.mark.parametrize("col", [5, 700, 1663])
def test_not_positive_definite_reports_column(gpu, col):
    n = 1700
    A = spd(n, seed=3)
    A[col, col] = -1.0
    _, info_o = oracle.cholesky(A)
    assert info_o == col + 1
    for own in (6, 2, 1, 0):
        for la in (0, 1):
            _, _, info = mi_ba.dense_cholesky(A, panel=512, lookahead=la, own_diag=own)
            assert info == col + 1, (own, la, info)


def test_concurrent_factorisations_share_nothing(gpu):
    mats = [spd(1700, seed=s) for s in (11, 12, 13, 14)]
    serial = [mi_ba.dense_cholesky(A, np.ones(1700)) for A in mats]
    out = [None] * len(mats)

    def run(k):
        out[k] = mi_ba.dense_cholesky(mats[k], np.ones(1700))

    ts = [threading.Thread(target=run, args=(k,)) for k in range(len(mats))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    for k in range(len(mats)):
        assert np.array_equal(out[k][0], serial[k][0]) and np.array_equal(out[k][1], serial[k][1])


def test_two_contexts_two_threads(gpu):
    """Two resident contexts solving at once on one device (each owns its
    look-ahead side stream, rocBLAS handles and events) reach the results of
    the same solves run one after the other."""
    scenes = [mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 120, 3000, track_length=6,
                                                      rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=s)).gauge()
              for s in (21, 22)]
    opts = mi_ba.default_options(max_num_iterations=6)

    def solve(sc):
        with mi_ba.Context(opts, sc.copy()) as ctx:
            return ctx.solve()

    serial = [solve(sc) for sc in scenes]
    out = [None, None]

    def run(k):
        out[k] = solve(scenes[k])

    ts = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    for a, b in zip(out, serial):
        assert a.num_successful_steps == b.num_successful_steps
        assert a.num_unsuccessful_steps == b.num_unsuccessful_steps
        assert abs(a.final_cost - b.final_cost) <= 1e-9 * b.final_cost


def test_lm_solve_variants(gpu):
    """The sync-free sweeps (default), the per-block-column sweeps and the
    recursive rocBLAS dtrsv / dgemv solve drive the same LM (nf = 1593,
    ragged last block)."""
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 200, 20000, track_length=8,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=5)).gauge()
    opts = mi_ba.default_options(max_num_iterations=10)
    res = []
    for v in (0, 1, 2):
        with mi_ba.Context(opts, sc.copy()) as ctx:
            ctx.set_tuning("cholesky_solve", v)
            res.append(ctx.solve())
    b = res[-1]
    for a in res[:-1]:
        assert (a.num_successful_steps, a.num_unsuccessful_steps) == (b.num_successful_steps, b.num_unsuccessful_steps)
        assert abs(a.final_cost - b.final_cost) <= 1e-9 * b.final_cost


@pytest.mark.parametrize("images", [200])
def test_lm_lookahead_on_off(gpu, images):
    """LM at nf = 1593 (C2 shape, 4 panels): look-ahead on/off give the same
    steps and final cost (within the run-to-run spread of the atomics-based
    normal-equation build)."""
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, images, 20000, track_length=8,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=4)).gauge()
    opts = mi_ba.default_options(max_num_iterations=10)
    res = []
    for la in (0, 1):
        with mi_ba.Context(opts, sc.copy()) as ctx:
            ctx.set_tuning("cholesky_lookahead", la)
            res.append(ctx.solve())
    a, b = res
    assert a.num_successful_steps == b.num_successful_steps
    assert a.num_unsuccessful_steps == b.num_unsuccessful_steps
    assert abs(a.final_cost - b.final_cost) <= 1e-9 * b.final_cost


def test_factor_at_c4_size_matches_lapack(gpu):
    """nf = 11 993, the C4 reduced camera system (998 * 6 + 5 + 1000 * 6): the
    default factorisation the bench times (24 panels of 512, one-launch panel
    factor, look-ahead, sync-free sweeps) on a random DENSE SPD matrix against
    LAPACK dpotrf: max|dL| <= 1e-12 * max|L|, solve within 1e-10 of LAPACK's."""
    from scipy.linalg import cho_factor, cho_solve
    n = 11993
    rng = np.random.default_rng(n)
    G = rng.standard_normal((n, 1024))
    A = G @ G.T / 1024.0 + np.diag(rng.uniform(0.5, 2.0, n))
    del G
    b = rng.standard_normal(n)
    L, x, info = mi_ba.dense_cholesky(A, b)
    assert info == 0
    c, low = cho_factor(A, lower=True, check_finite=False)
    L_ref = np.tril(c)
    scale = np.abs(L_ref).max()
    assert np.abs(L - L_ref).max() <= 1e-12 * scale
    x_ref = cho_solve((c, low), b, check_finite=False)
    assert np.abs(x - x_ref).max() <= 1e-10 * np.abs(x_ref).max()


def test_lm_tile_factor_and_publish(gpu):
    """The panel factor's 64x64 tile factor (block-column register sweeps
    with rsq (2) or sqrt + divide (1) pivots) and its publish (write-through
    sc1 stores drained before the flag vs plain stores + __threadfence())
    drive the same LM (nf = 1593: 4 panels), all four combinations (the
    non-default ones are in the tools-only A/B build)."""
    if not mi_ba.ab_build():
        pytest.skip("tile factor 1 / plain-store publish: tools build only (MI_BA_LIB=ab)")
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 200, 20000, track_length=8,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=6)).gauge()
    opts = mi_ba.default_options(max_num_iterations=10)
    res = []
    for tf in (2, 1, 3, 4, 5, 6):
        for wt in ((1, 0) if tf <= 2 else (1,)):
            with mi_ba.Context(opts, sc.copy()) as ctx:
                ctx.set_tuning("cholesky_tile_factor", tf)
                ctx.set_tuning("cholesky_write_through", wt)
                res.append(ctx.solve())
    b = res[0]
    for a in res[1:]:
        assert (a.num_successful_steps, a.num_unsuccessful_steps) == (b.num_successful_steps, b.num_unsuccessful_steps)
        assert abs(a.final_cost - b.final_cost) <= 1e-9 * b.final_cost


@pytest.mark.parametrize("images", [200, 1000])
def test_lm_handoff_variants_bitwise(gpu, images):
    """The panel factor's hand-off waits (every wave acquires / one wave
    acquires for the workgroup / one wave polls and the tiles are read by sc1
    loads, with or without the next stage's tiles loaded during the current
    GEMM) and the sweeps' sc1 hand-offs (no fences) change only
    synchronisation: the same LM bit for bit (deterministic sums; nf = 1593,
    4 panels, ragged last sweep block; nf = 7993, 16 panels, at C4's panel
    count order).  Non-default combinations: tools-only A/B build."""
    if not mi_ba.ab_build():
        pytest.skip("hand-off variants: tools build only (MI_BA_LIB=ab)")
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, images, 100 * images, track_length=8,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=6)).gauge()
    opts = mi_ba.default_options(max_num_iterations=10 if images <= 200 else 4)
    res = []
    for wm, sc1 in ((2, 1), (0, 0), (1, 0), (2, 0), (3, 1)):
        b = sc.copy()
        with mi_ba.Context(opts, b) as ctx:
            ctx.set_tuning("cholesky_panel_wait", wm)
            ctx.set_tuning("cholesky_solve_sc1", sc1)
            s = ctx.solve()
            ctx.writeback()
        res.append((s.num_successful_steps, s.num_unsuccessful_steps, s.final_cost,
                    b.qvec.tobytes(), b.tvec.tobytes(), b.xyz.tobytes(), b.camera_params.tobytes()))
    for r in res[1:]:
        assert r == res[0]


def test_lm_split_panel_bitwise(gpu):
    """Split panel (cholesky_split_panel_cols): the diagonal block's row tiles
    and the rows below it in two launches, one after the other, on the
    look-ahead stream (the same kernel, flags and GEMMs) — the LM bit for bit
    the one-launch panel's (nf = 1593, 4 panels; split for the first 1024
    columns and for all of them).  Tools build (measured slower)."""
    if not mi_ba.ab_build():
        pytest.skip("split panel: tools build only (MI_BA_LIB=ab)")
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 200, 20000, track_length=8,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=6)).gauge()
    opts = mi_ba.default_options(max_num_iterations=10)
    res = []
    for cols in (0, 1024, 100000):
        b = sc.copy()
        with mi_ba.Context(opts, b) as ctx:
            ctx.set_tuning("cholesky_split_panel_cols", cols)
            s = ctx.solve()
            ctx.writeback()
        res.append((s.num_successful_steps, s.num_unsuccessful_steps, s.final_cost,
                    b.qvec.tobytes(), b.tvec.tobytes(), b.xyz.tobytes(), b.camera_params.tobytes()))
    for r in res[1:]:
        assert r == res[0]


@pytest.mark.parametrize("images", [40, 120, 200])
def test_lm_look_ahead_on_side_stream_bitwise(gpu, images):
    """The look-ahead dgemm on the panel's side stream
    (cholesky_la_side_from 0: from the second panel on; 1024: from column
    1024) instead of the caller's stream (-1): the same GEMMs on the same
    operands, ordered by the side stream and the previous update's first
    block-column event — the LM bit for bit the default's (nf = 313: one
    panel, 953: two, 1593: four).  With the trailing update's first block
    column only one panel wide (cholesky_rest_first_panel 1) the dgemms
    cover the same entries in other column ranges: bitwise as well (tools
    build)."""
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, images, 100 * images, track_length=8,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=6)).gauge()
    opts = mi_ba.default_options(max_num_iterations=10)
    res = []
    firsts = (0, 1) if mi_ba.ab_build() else (0,)  # rest_first_panel 1: tools build
    for frm, first in [(f, x) for x in firsts for f in (-1, 0, 1024, 0)]:
        b = sc.copy()
        with mi_ba.Context(opts, b) as ctx:
            ctx.set_tuning("cholesky_la_side_from", frm)
            ctx.set_tuning("cholesky_rest_first_panel", first)
            s = ctx.solve()
            ctx.writeback()
        res.append((s.num_successful_steps, s.num_unsuccessful_steps, s.final_cost,
                    b.qvec.tobytes(), b.tvec.tobytes(), b.xyz.tobytes(), b.camera_params.tobytes()))
    assert res[0][0] >= 2
    for r in res[1:]:
        assert r == res[0]


def test_lm_split_tail(gpu):
    """Split tail (cholesky_split_tail_cols, tools build): the next panel's
    block column updated in two dgemms and the panel's below-diagonal rows as
    a second launch on a second side stream (or on the second trailing-update
    stream, cholesky_split_tail_rest), over the last 1024 / all columns
    (nf = 1593: 4 panels): the same LM steps as the one-launch panels, final
    cost within 1e-9 (different dgemm shapes sum in a different order), and
    bit for bit repeatable."""
    if not mi_ba.ab_build():
        pytest.skip("split tail: tools build only (MI_BA_LIB=ab)")
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 200, 20000, track_length=8,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=6)).gauge()
    opts = mi_ba.default_options(max_num_iterations=10)
    res = []
    for cols, rest in ((0, 0), (1024, 0), (100000, 0), (100000, 0), (100000, 1)):
        with mi_ba.Context(opts, sc.copy()) as ctx:
            ctx.set_tuning("cholesky_split_tail_cols", cols)
            ctx.set_tuning("cholesky_split_tail_rest", rest)
            res.append(ctx.solve())
    b = res[0]
    for a in res[1:]:
        assert (a.num_successful_steps, a.num_unsuccessful_steps) == (b.num_successful_steps, b.num_unsuccessful_steps)
        assert abs(a.final_cost - b.final_cost) <= 1e-9 * b.final_cost
    assert res[2].final_cost == res[3].final_cost


def test_lm_gemm_solution(gpu):
    """The trailing update through rocblas_gemm_ex with an explicit Tensile
    solution index (cholesky_gemm_solution; an index the shape does not accept
    falls back to the default) drives the same LM as rocBLAS's default
    dgemm (nf = 1593)."""
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 200, 20000, track_length=8,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=6)).gauge()
    opts = mi_ba.default_options(max_num_iterations=10)
    res = []
    for sol in (0, -624952238, -624952224, 12345):
        with mi_ba.Context(opts, sc.copy()) as ctx:
            ctx.set_tuning("cholesky_gemm_solution", sol)
            res.append(ctx.solve())
    b = res[0]
    for a in res[1:]:
        assert (a.num_successful_steps, a.num_unsuccessful_steps) == (b.num_successful_steps, b.num_unsuccessful_steps)
        assert abs(a.final_cost - b.final_cost) <= 1e-9 * b.final_cost


def test_lm_schur_pair_orders(gpu):
    """The explicit Schur build's pair tiles in first-image order with the
    XCD-striped mapping (schur_pairs_variant 0), in image-block order with
    dispatch-order mapping (4, blocks of 8 and 64 images), the JG records
    with two pairs per MFMA (6: Z_a Z_b' = J_f,a' (G_a' G_b) J_f,b) and
    XCD-interleaved by first image with padding tiles (5) and the Z rows
    formed in the pair kernel from J and Linv (7) drive the same LM:
    the same S up to the order of the float atomics (nf = 1593)."""
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 200, 20000, track_length=8,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=6)).gauge()
    opts = mi_ba.default_options(max_num_iterations=10)
    res = []
    orders = ((0, 32), (4, 8), (4, 64), (6, 8)) + (((5, 8), (7, 8), (8, 8), (9, 8)) if mi_ba.ab_build() else ())
    for var, blk in orders:
        with mi_ba.Context(opts, sc.copy()) as ctx:
            ctx.set_tuning("schur_pairs_variant", var)
            ctx.set_tuning("schur_block_images", blk)
            res.append(ctx.solve())
    b = res[0]
    for a in res[1:]:
        assert (a.num_successful_steps, a.num_unsuccessful_steps) == (b.num_successful_steps, b.num_unsuccessful_steps)
        assert abs(a.final_cost - b.final_cost) <= 1e-9 * b.final_cost


@pytest.mark.parametrize("images", [40, 200])
def test_lm_fused_forward_solve(gpu, images):
    """The forward solve L y = b carried through the factorisation in S's
    spare row (cholesky_fused_rhs 1, the default: one backward sweep left)
    drives the same LM as the two separate sweeps (0), at one panel (nf = 313)
    and several (nf = 1593)."""
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, images, 100 * images, track_length=8,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=7)).gauge()
    opts = mi_ba.default_options(max_num_iterations=10)
    res = []
    for fused in (1, 0):
        with mi_ba.Context(opts, sc.copy()) as ctx:
            ctx.set_tuning("cholesky_fused_rhs", fused)
            res.append(ctx.solve())
    a, b = res
    assert (a.num_successful_steps, a.num_unsuccessful_steps) == (b.num_successful_steps, b.num_unsuccessful_steps)
    assert abs(a.final_cost - b.final_cost) <= 1e-9 * b.final_cost
    assert a.final_cost < a.initial_cost


@pytest.mark.parametrize("schedule", [dict(head_panel=1024, head_cols=1024), dict(tail_panel=256, tail_cols=768),
                                      dict(head_panel=768, head_cols=700, tail_panel=128, tail_cols=300),
                                      dict(split_cus=32, split_cols=1024), dict(split_cus=200, split_cols=1593),
                                      dict(head_own_diag=2, head_own_cols=1024),
                                      dict(rest_streams=2, rest_update=0), dict(rest_streams=4, rest_update=0),
                                      dict(rest_streams=3), dict(rest_streams=2)])
def test_lm_panel_schedule(gpu, schedule):
    """Non-uniform panel schedules (cholesky_head_panel / _head_cols /
    _tail_panel / _tail_cols: 1024-wide one-launch panels of 16 column tiles,
    narrower ones at the end) drive the same LM as the uniform 512-wide
    panels (nf = 1593), as do the split head (cholesky_split_cus / _cols:
    the panel factor and the trailing dgemm on disjoint CU sets) and the
    two-kernel diagonal factor + dtrsm for the head panels
    (cholesky_head_own_diag / _cols) and the trailing update's block columns
    over several streams (cholesky_rest_streams), with and
    without the look-ahead (S itself differs
    between runs in the order of the Schur build's float atomics).  The
    baseline is the single-stream trailing update (rest_streams 1), so the
    default two-stream update is compared with it too."""
    if any(k in schedule for k in ("split_cus", "head_own_diag")) and not mi_ba.ab_build():
        pytest.skip("split head / head panel kind: tools build only (MI_BA_LIB=ab)")
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 200, 20000, track_length=8,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=6)).gauge()
    opts = mi_ba.default_options(max_num_iterations=10)
    res = []
    for keys in (dict(rest_streams=1), schedule, dict(schedule, lookahead=0)):
        with mi_ba.Context(opts, sc.copy()) as ctx:
            for k, v in keys.items():
                ctx.set_tuning("cholesky_" + k, v)
            res.append(ctx.solve())
    b = res[0]
    for a in res[1:]:
        assert (a.num_successful_steps, a.num_unsuccessful_steps) == (b.num_successful_steps, b.num_unsuccessful_steps)
        assert abs(a.final_cost - b.final_cost) <= 1e-9 * b.final_cost
