"""The RCCL path of the multi-rank LM (mi_ba_context_set_comm), on one GPU.

The driver's multi-GPU bench is the only place several GPUs are available, so
the RCCL code path is pinned here at world 1 and its failure handling with a
peer that never arrives:

  * a 1-rank communicator routes every sum of the multi-rank LM (model / trial
    costs, the f-blocks, S in 512-row bands on the exact path, one nf-vector
    per Schur product on the PCG path, the callback decisions) through
    ncclAllReduce; C2 solved that way takes the communicator-less solve's
    steps bitwise (the camera-side sums are flushed in a fixed order, so the
    LM is reproducible run to run: tests/test_determinism.py);
  * a collective that does not complete by the deadline ("comm_timeout_ms";
    forced with the "comm_stall_ms" hook, a kernel holding the stream ahead of
    each collective as a missing peer would) aborts the communicator and the
    solve returns MI_BA_ERR_HIP instead of hanging;
  * a communicator set-up whose peer never joins (world 2, rank 1 absent)
    returns MI_BA_ERR_HIP at the deadline, and the context stays usable as a
    single-rank context.

Reference: the reduced camera system solve of BundleAdjuster::Solve
(bundle_adjustment.cc:281-286); SURVEY 8e (point-sharded LM, RCCL all-reduce).
"""
import os
import subprocess
import sys
import time

import numpy as np
import pytest

import mi_ba

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def c2_scene():
    return mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 200, 50_000, track_length=10,
                                                   rotation_range=0.05, extra=(0.05, 0, 0, 0))).gauge()


def _solve(opts, sc, comm):
    with mi_ba.Context(opts, sc) as ctx:
        if comm:
            ctx.set_comm(0, 1, mi_ba.comm_unique_id())
        s = ctx.solve()
        ctx.writeback()
    return s


@pytest.mark.parametrize("solver", ["exact", "pcg"])
def test_one_rank_rccl_matches_commless_bitwise(gpu, solver):
    """With the camera-side sums flushed per image / camera in a fixed order
    (owner_flush_kernel, the Schur pair flush, the semantic pair sums), the
    LM is bitwise reproducible, and a 1-rank communicator (every sum of the
    multi-rank LM through ncclAllReduce) takes exactly the communicator-less
    solve's steps: same step and CG counts, costs and parameters bitwise."""
    sc = c2_scene()
    kw = dict(max_num_iterations=6)
    if solver == "pcg":
        kw.update(linear_solver_type=mi_ba.SOLVER_ITERATIVE_SCHUR)  # default eta, as bench.py at N > 1
    else:
        kw.update(linear_solver_type=mi_ba.SOLVER_DENSE_SCHUR)
    a, b = sc.copy(), sc.copy()
    s0 = _solve(mi_ba.default_options(**kw), a, comm=False)
    s1 = _solve(mi_ba.default_options(**kw), b, comm=True)
    assert s1.num_successful_steps >= 3
    assert (s1.num_successful_steps, s1.num_unsuccessful_steps) == (s0.num_successful_steps, s0.num_unsuccessful_steps)
    assert s1.num_linear_solver_iterations == s0.num_linear_solver_iterations
    assert s1.initial_cost == s0.initial_cost
    assert s1.final_cost == s0.final_cost
    for key in ("qvec", "tvec", "xyz", "camera_params"):
        assert np.array_equal(getattr(a, key), getattr(b, key)), key


def test_stalled_collective_aborts_instead_of_hanging(gpu):
    sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 10, 300, track_length=4,
                                                 rotation_range=0.05, extra=(0.05, 0, 0, 0), seed=3)).gauge()
    with mi_ba.Context(mi_ba.default_options(max_num_iterations=3), sc.copy()) as ctx:
        ctx.set_comm(0, 1, mi_ba.comm_unique_id())
        ctx.set_tuning("comm_timeout_ms", 300)
        ctx.set_tuning("comm_stall_ms", 3000)
        t0 = time.perf_counter()
        with pytest.raises(mi_ba.MiBaError) as e:
            ctx.solve()
        dt = time.perf_counter() - t0
        assert e.value.status == mi_ba.ERR_HIP
        assert dt < 2.5, dt  # the deadline ended the wait, not the stall
    # the same context without the stall: the communicator path solves
    with mi_ba.Context(mi_ba.default_options(max_num_iterations=3), sc.copy()) as ctx:
        ctx.set_comm(0, 1, mi_ba.comm_unique_id())
        ctx.set_tuning("comm_timeout_ms", 300)
        assert ctx.solve().num_successful_steps >= 1


def test_missing_peer_at_setup_returns_error(gpu):
    # in a child process: a communicator set-up that RCCL could not abort
    # would otherwise hold the test runner
    p = subprocess.run([sys.executable, os.path.join(HERE, "comm_missing_peer.py")], capture_output=True, text=True,
                       timeout=180)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "missing peer: ERR_HIP" in p.stdout, p.stdout
    # RCCL 2.27's init call blocks in its bootstrap while the peer is missing
    # (no timeout, non-blocking config or not): the helper stays inside it,
    # reported, and the context solves single-rank regardless
    assert "set-up helpers still running: 1" in p.stdout, p.stdout
    assert "single-rank solve after the failed set-up" in p.stdout, p.stdout
