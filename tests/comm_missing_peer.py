"""Child process of tests/test_comm.py: rank 0 of a 2-rank RCCL communicator
whose rank 1 never joins.  mi_ba_context_set_comm must return MI_BA_ERR_HIP
at the "comm_timeout_ms" deadline, after which the context still solves as a
single-rank context."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd"))
import mi_ba  # noqa: E402

sc = mi_ba.generate_scene(mi_ba.synth_config(mi_ba.SIMPLE_RADIAL, 10, 300, track_length=4, rotation_range=0.05,
                                             extra=(0.05, 0, 0, 0), seed=3)).gauge()
with mi_ba.Context(mi_ba.default_options(max_num_iterations=3), sc.copy()) as ctx:
    ctx.set_tuning("comm_timeout_ms", 3000)
    t0 = time.perf_counter()
    try:
        ctx.set_comm(0, 2, mi_ba.comm_unique_id())
        print("missing peer: joined (unexpected)")
        sys.exit(1)
    except mi_ba.MiBaError as e:
        dt = time.perf_counter() - t0
        name = "ERR_HIP" if e.status == mi_ba.ERR_HIP else f"status {e.status}"
        print(f"missing peer: {name} after {dt:.2f} s", flush=True)
        if e.status != mi_ba.ERR_HIP or dt > 30:
            sys.exit(1)
    # the abandoned set-up's helper is still inside RCCL's init call (its
    # bootstrap waits for the peer with no timeout): reported, not joined
    pending = mi_ba.comm_pending_setups()
    print(f"set-up helpers still running: {pending}", flush=True)
    if pending > 1:
        sys.stdout.flush()
        os._exit(1)
    s = ctx.solve()
    print(f"single-rank solve after the failed set-up: {s.num_successful_steps} steps", flush=True)
    ok = s.num_successful_steps >= 1
# RCCL's own bootstrap threads may outlive the aborted communicator: end the
# process without waiting for them
sys.stdout.flush()
os._exit(0 if ok else 1)
