#!/usr/bin/env python3
"""bench.py — residuals+Jacobians/sec of the semantic-BA hot path on MI355X.

A step is one full linearization of the BASELINE.json workload already
resident in HBM: every reprojection residual block (residual + loss-corrected
tangent Jacobian, written to HBM) and every semantic sample (residual +
29-point CENTRAL numeric-diff Jacobian, reduced into the per-pair J'J / J'r
blocks; the stencil is evaluated point by point for the samples whose
Jacobian the flat test cannot prove to be exactly zero, ~9 % at C4, with
results bitwise equal to evaluating it everywhere) — mi_ba_linearize on the
context's stream.  The point and camera
normal-equation blocks are reduced by the LM's own passes (timed in the
BA-iteration figures), not inside the step.

value = (reprojection blocks + semantic samples, all ranks) * steps / max-over-
ranks wall time of the timed steps.  Multi-GPU: the linearization shards by
point blocks (with all their observations) and image pairs and has no
data-path collective, so the timed region needs none.  Default at N > 1:
--scaling strong, the one C4 problem split across the ranks (BASELINE's C5);
--scaling weak gives every rank a C4-sized shard of its own (labelled).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config C4]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd")
sys.path.insert(0, PKG)
import mi_ba  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]

OPENCV_EXTRA = (-0.1, 0.01, 1e-4, -1e-4)
CONFIGS = {
    "C2": dict(model=mi_ba.SIMPLE_RADIAL, images=200, points=50_000, track=10, extra=(0.05, 0, 0, 0),
               semantic=None, desc="200 cams / 50k points / 500k obs, SIMPLE_RADIAL, geometric"),
    "C3": dict(model=mi_ba.SIMPLE_RADIAL, images=200, points=50_000, track=10, extra=(0.05, 0, 0, 0),
               semantic=dict(step=10, pairs_per_image=2, size=1000),
               desc="200 cams / 50k points / 500k obs, SIMPLE_RADIAL, geometric + semantic (4.0M samples)"),
    "C4": dict(model=mi_ba.OPENCV, images=1000, points=1_000_000, track=10, extra=OPENCV_EXTRA,
               semantic=dict(step=20, pairs_per_image=2, size=1000),
               desc="1k cams / 1M points / 10M obs, OPENCV, semantic BA (5.0M samples)"),
}
# Algorithmic bytes per reprojection block: 24 (obs) + 24/L
# (point) + 16 (residual) + 16*(9+c) (tangent Jacobian), c = refined intrinsics
# with the default refine flags: SIMPLE_RADIAL 2, OPENCV 6.
CAM_TANGENT = {mi_ba.SIMPLE_PINHOLE: 1, mi_ba.PINHOLE: 2, mi_ba.SIMPLE_RADIAL: 2, mi_ba.RADIAL: 3, mi_ba.OPENCV: 6}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def pmc_traffic(config, kernel_prefix):
    """HBM bytes per launch of a kernel from the newest committed PMC summary
    (profiles/<round>_<config>_traffic.json, written by tools/summarize_profile.py
    from separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this bench)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{config.lower()}_traffic.json")))
    for f in reversed(files):
        d = json.load(open(f))
        for name, v in d.get("kernels", {}).items():
            if name.startswith(kernel_prefix):
                return v["hbm_bytes"], os.path.relpath(f, ROOT)
    return None, None


FP64_PEAK_TFS = 78.6  # MI355X vector FP64 (MI355X_MICROARCH.md)


def semantic_pmc(config):
    """FP64 operations and HBM bytes per launch of the semantic kernel from the
    newest committed PMC summary (profiles/<round>_<config>_semantic_pmc.json,
    tools/pmc_semantic.sh + tools/summarize_pmc_semantic.py)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{config.lower()}_semantic_pmc.json")))
    if not files:
        return None, None, None
    d = json.load(open(files[-1]))
    return d.get("fp64_ops_per_launch"), d.get("hbm_bytes_per_launch"), os.path.relpath(files[-1], ROOT)


def bytes_per_block(model, track):
    return 24 + 24.0 / track + 16 + 16 * (9 + CAM_TANGENT[model])


def build_shard(cfg, rank, world, scaling="weak"):
    """This rank's shard.  weak: every rank owns a full config-sized block of
    points (synthetic scene seeded with the rank; the per-GPU work is fixed as
    ranks are added).  strong: one scene (seed 0) whose points, with all their
    observations, and image pairs are split into contiguous rank ranges."""
    weak = scaling == "weak"
    c = mi_ba.synth_config(cfg["model"], cfg["images"], cfg["points"], track_length=cfg["track"],
                           rotation_range=0.05, extra=cfg["extra"], seed=rank if weak else 0)
    full = mi_ba.generate_scene(c).gauge()
    if weak:
        rank, world = 0, 1
    P = full.num_points
    p0, p1 = P * rank // world, P * (rank + 1) // world
    m = (full.obs_point >= p0) & (full.obs_point < p1)
    sc = full
    if world > 1:
        sc.obs_xy, sc.obs_image, sc.obs_point = full.obs_xy[m], full.obs_image[m], full.obs_point[m]
    sem = None
    if cfg["semantic"]:
        s = cfg["semantic"]
        I = cfg["images"]
        pairs = np.array([(i, (i + d) % I) for i in range(I) for d in range(1, s["pairs_per_image"] + 1)], np.int32)
        K = len(pairs)
        pairs = pairs[K * rank // world:K * (rank + 1) // world]
        H = W = s["size"]
        need = np.unique(pairs.reshape(-1))
        depth = np.zeros((I, H, W), np.float32)
        label = np.zeros((I, H, W), np.float32)
        sub = mi_ba.Scene(sc.camera_model, sc.camera_params, sc.qvec[need], sc.tvec[need], sc.image_camera[need],
                          sc.xyz[:1], sc.obs_xy[:0], sc.obs_image[:0], sc.obs_point[:0])
        d_sub, l_sub = mi_ba.render_semantic(sub, H, W, plane_z=1.0, cell=0.1)
        depth[need] = d_sub
        label[need] = l_sub
        del d_sub, l_sub
        sem = mi_ba.SemanticInput(depth, label, pairs, pixel_step=s["step"])
    return sc, sem


def host_cpu():
    """CPU model, logical CPUs of the machine and of this process's affinity mask."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    return model, os.cpu_count() or 1, affinity


def cpu_threads():
    """Threads for the CPU baseline: the CPUs this process may use.  On the
    GPU boxes the job's CPU share is exported as OMP_NUM_THREADS (16 per GPU)
    while nproc reports the whole host; the share is what the baseline gets."""
    _, nproc, affinity = host_cpu()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(affinity, share) if share > 0 else affinity


def cpu_ba_iteration(iters=3):
    """CPU BA-iteration wall time of the oracle's LM (dense Schur, 'port',
    not Ceres) on C2, and the GPU's on the same problem."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    c = CONFIGS["C2"]
    sc = mi_ba.generate_scene(mi_ba.synth_config(c["model"], c["images"], c["points"], track_length=c["track"],
                                                 rotation_range=0.05, extra=c["extra"])).gauge()
    opts = mi_ba.default_options(max_num_iterations=iters)
    t0 = time.perf_counter()
    s0 = oracle.solve(mi_ba.default_options(max_num_iterations=0), sc.copy())
    t_setup = time.perf_counter() - t0
    t0 = time.perf_counter()
    s = oracle.solve(opts, sc.copy())
    wall = time.perf_counter() - t0 - t_setup
    its = max(1, s.num_successful_steps + s.num_unsuccessful_steps)
    with mi_ba.Context(opts, sc.copy()) as ctx:  # solve time only (context setup excluded, as for the CPU)
        g = ctx.solve()
    g_its = max(1, g.num_successful_steps + g.num_unsuccessful_steps)
    return {"workload": "C2: 200 cams / 50k points / 500k obs, SIMPLE_RADIAL, exact Schur LM",
            "cpu_ms": 1e3 * wall / its, "cpu_kind": "port (oracle/ C++/OpenMP dense-Schur LM, not Ceres)",
            "gpu_ms": 1e3 * g.total_time_in_seconds / g_its, "iterations": its,
            "cpu_final_cost": s.final_cost, "gpu_final_cost": g.final_cost}


def cpu_baseline(opts, sc, sem, cfg, nb, ns):
    """The CPU restatement (oracle, 'port') timed on this host on a bounded
    sample of the same workload, at 1 thread and at the job's CPU share
    (OMP_NUM_THREADS = 16 on the GPU boxes; `value`).  The host has more
    CPUs (affinity_cpus) than the share this job may load — the pool's rule is
    to size worker pools to the share — so the whole-host figure is the
    share's rate scaled linearly by affinity_cpus / cores (an upper bound:
    memory bandwidth does not scale with threads), reported as an
    extrapolation, not a measurement."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    threads = cpu_threads()

    def rates(nthreads, geo_blocks, sem_samples):
        t_geo, done_geo = oracle.reproj_throughput(opts, sc, geo_blocks, 1, nthreads)
        r_geo = done_geo / t_geo
        r_sem, done_sem = None, 0
        if sem is not None and ns:
            t_sem, done_sem = oracle.semantic_throughput(opts, sc, sem, sem_samples, nthreads)
            r_sem = done_sem / t_sem
        total = nb / r_geo + (ns / r_sem if r_sem else 0.0)
        return (nb + ns) / total, r_geo, r_sem, done_geo, done_sem

    # the whole workload at the share (~1.5 s wall x 16 threads); a bounded
    # sample single-threaded
    value, rate_geo, rate_sem, done_geo, done_sem = rates(threads, nb, ns)
    one, one_geo, one_sem, d1g, d1s = rates(1, min(nb, 500_000), min(ns, 100_000))
    model, nproc, affinity = host_cpu()
    sample = f"{done_geo} reprojection blocks" + (f" + {done_sem} semantic samples" if done_sem else "")
    return {"value": value, "unit": "residual_blocks/s", "cores": threads, "kind": "port",
            "sample": sample + " of the same workload at `cores` threads (1 thread: " +
                      f"{d1g} blocks" + (f" + {d1s} samples" if d1s else "") +
                      "), oracle/ CPU restatement (C++/OpenMP, f64), not Ceres",
            "reproj_blocks_per_s": rate_geo, "semantic_samples_per_s": rate_sem,
            "single_thread_value": one, "single_thread_reproj_blocks_per_s": one_geo,
            "single_thread_semantic_samples_per_s": one_sem,
            "parallel_efficiency": value / (one * threads) if one else None,
            "whole_host_extrapolated_value": value * affinity / max(1, threads),
            "whole_host_note": "linear extrapolation of the share's rate to affinity_cpus threads (not measured: "
                               "the job's CPU share is `cores`); an upper bound",
            "cpu_model": model, "host_nproc": nproc, "affinity_cpus": affinity,
            "threads_note": "threads = the job's CPU share (OMP_NUM_THREADS on the GPU box), capped by the affinity mask"}


def roofline_semantic(config, ns, avg_ms):
    """The semantic linearization (two-pass route: flat pass + deferred-sample
    pass, timed together; HIP events on the context stream) against both
    roofs, on ALGORITHMIC work:
      * HBM: SURVEY 8d's 128 B per sample (16 sample in, 8 compulsory raster
        gather, 8 residual + 96 tangent-Jacobian row out — the J-materialising
        definition, kept although the product reduces the rows into per-pair
        J'J / J'r blocks instead of writing them) x samples / time;
      * FP64: the PMC FP64 operation count per linearization (ADD/MUL/TRANS 1,
        FMA 2, x 64 lanes) / time, against 78.6 TF/s.
    `bound` names the roof with the larger fraction; `achieved` / `peak` /
    `unit` / `frac` are that roof's.  The measured (PMC) HBM traffic is
    `traffic` only: it is not the numerator of any fraction (a kernel that
    re-reads would otherwise score higher)."""
    flops, hbm, src = semantic_pmc(config)
    if avg_ms <= 0 or not ns:
        return None
    t = avg_ms * 1e-3
    alg = 128.0 * ns
    f_hbm = alg / t / 1e9 / HBM_PEAK_GBS
    f_fp64 = flops / t / 1e12 / FP64_PEAK_TFS if flops else 0.0
    hbm_bound = f_hbm >= f_fp64
    return {"kernel": "semantic_flat+semantic_deferred", "bound": "hbm" if hbm_bound else "fp64",
            "unit": "GB/s" if hbm_bound else "TFLOP/s",
            "peak": HBM_PEAK_GBS if hbm_bound else FP64_PEAK_TFS,
            "achieved": alg / t / 1e9 if hbm_bound else flops / t / 1e12,
            "frac": f_hbm if hbm_bound else f_fp64,
            "algorithmic_bytes_per_sample": 128, "algorithmic_bytes_per_launch": alg,
            "hbm_algorithmic_GBs": alg / t / 1e9, "hbm_algorithmic_frac": f_hbm,
            "fp64_achieved_TFs": flops / t / 1e12 if flops else None, "fp64_frac": f_fp64 if flops else None,
            "fp64_ops_per_launch": flops,
            "traffic": hbm, "traffic_unit": "bytes/launch (PMC FETCH_SIZE x 2 + WRITE_SIZE; not a numerator)",
            "traffic_bytes_per_sample": hbm / ns if hbm else None,
            "traffic_GBs": hbm / t / 1e9 if hbm else None,
            "samples_per_launch": ns, "avg_launch_ms": avg_ms, "pmc_source": src}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # 30: the first ~20 steps after the context's setup run slower (0.84 vs
    # 0.78 ms at C4, profiles/r6z_step_timing_probe.jsonl) — the timed steps
    # start in the steady state
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--config", default="C4", choices=sorted(CONFIGS))
    ap.add_argument("--lm-iters", type=int, default=3, help="LM iterations for the BA-iteration wall time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--lm-solver", default=None, choices=["exact", "iterative"],
                    help="reduced camera system of the BA-iteration figure: exact (dense Schur + Cholesky, "
                         "the 1-GPU default) or iterative (ITERATIVE_SCHUR + SCHUR_JACOBI: one nf-vector "
                         "all-reduce per CG product, the default at N > 1, where an exact solve would have "
                         "every rank factor the same summed S)")
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="strong (default at N > 1): the one config problem split across the ranks (C4 split "
                         "this way is BASELINE's C5); weak: a config-sized shard per rank")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.scaling is None:
        args.scaling = "strong" if world > 1 else "weak"  # N = 1: both are the whole config
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ap_backend = os.environ.get("MI_BA_BENCH_BACKEND", "nccl")  # nccl == RCCL on ROCm; gloo for 1-GPU rehearsals
    dist = None
    device = local_rank
    if world > 1:
        import torch
        import torch.distributed as tdist
        device = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(device)
        tdist.init_process_group(ap_backend)
        dist = tdist

    def barrier():
        if dist is not None:
            dist.barrier()

    def allreduce_max(v):
        if dist is None:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64, device=f"cuda:{device}" if ap_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def allreduce_sum(v):
        if dist is None:
            return v
        import torch
        t = torch.tensor([v], dtype=torch.float64, device=f"cuda:{device}" if ap_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    cfg = CONFIGS[args.config]
    t_setup = time.time()
    sc, sem = build_shard(cfg, rank, world, args.scaling)
    opts = mi_ba.default_options(device=device)
    ctx = mi_ba.Context(opts, sc, sem)
    nb, W, ns = ctx.dims()
    setup_s = time.time() - t_setup

    for _ in range(args.warmup):
        ctx.linearize()
    ctx.synchronize()
    ctx.set_timing(True)
    ctx.reset_kernel_times()
    barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.linearize()
    ctx.synchronize()
    t1 = time.perf_counter()
    barrier()
    dt = allreduce_max(t1 - t0)
    j_ms, j_n = ctx.kernel_time("reproj_jacobian")
    s_ms, s_n = ctx.kernel_time("semantic_jacobian")
    w_ms, w_n = ctx.kernel_time("input_warm")
    ctx.set_timing(False)
    # the linearization context is done: closed before the BA-iteration leg
    # (its idle streams otherwise share the LM context's hardware queues:
    # Cholesky 15.9 vs 14.7 ms, profiles/r4za_ab_cholesky_rest_streams_closed.jsonl)
    ctx.close()
    total_blocks = allreduce_sum(float(nb + ns))
    value = total_blocks * args.steps / dt

    # BA-iteration wall time: a few LM iterations on the same resident context
    lm = None
    if args.lm_iters > 0:
        # warm the LM path (lazy code-object loading of every LM kernel and of
        # rocSOLVER) on a small scene of the same model before timing it
        wc = mi_ba.synth_config(cfg["model"], 30, 300, track_length=5, rotation_range=0.05, extra=cfg["extra"])
        wsc = mi_ba.generate_scene(wc).gauge()
        wsem = None
        if sem is not None:
            wd, wl = mi_ba.render_semantic(wsc, 64, 64, cell=0.5)
            wsem = mi_ba.SemanticInput(wd, wl, np.array([(i, (i + 1) % 30) for i in range(30)], np.int32),
                                       pixel_step=8)
        with mi_ba.Context(mi_ba.default_options(device=device, max_num_iterations=2), wsc, wsem) as wctx:
            wctx.solve()
        lm_sc, lm_sem = sc, sem
        if world > 1:
            # C5: the one C4 problem point-sharded across the ranks, reduced camera
            # system summed over RCCL (xGMI) every LM iteration
            lm_sc, lm_sem = build_shard(cfg, rank, world, "strong")
        lm_solver = args.lm_solver or ("iterative" if world > 1 else "exact")
        ctx_lm = mi_ba.Context(mi_ba.default_options(
            device=device, max_num_iterations=args.lm_iters,
            linear_solver_type=mi_ba.SOLVER_ITERATIVE_SCHUR if lm_solver == "iterative" else mi_ba.SOLVER_DENSE_SCHUR),
            lm_sc, lm_sem)
        if world > 1:
            if ap_backend == "nccl":
                obj = [mi_ba.comm_unique_id() if rank == 0 else None]
                dist.broadcast_object_list(obj, src=0)
                ctx_lm.set_comm(rank, world, obj[0])
            else:
                sys.path.insert(0, os.path.join(ROOT, "tests"))
                import multirank_cases
                ctx_lm.set_host_reducer(rank, world, multirank_cases.gloo_reducer())
        ctx_lm.set_timing(True)
        barrier()
        s = ctx_lm.solve()
        its = max(1, s.num_successful_steps + s.num_unsuccessful_steps)
        lm = {"ba_iteration_ms": allreduce_max(1e3 * s.total_time_in_seconds / its), "iterations": its,
              "ba_iteration_workload": (((("C5 = " if args.config == "C4" else "") +
                                          f"{args.config} point-sharded across {world} ranks, S summed by ") +
                                         ("RCCL all-reduce" if ap_backend == "nccl" else "gloo host reducer"))
                                        if world > 1 else f"{args.config} on one GPU"),
              "lm_solver": ("ITERATIVE_SCHUR + SCHUR_JACOBI (nf-vector all-reduce per CG product)"
                            if lm_solver == "iterative" else "exact dense Schur + Cholesky"),
              "linear_solver_iterations": s.num_linear_solver_iterations,
              "initial_cost": s.initial_cost, "final_cost": s.final_cost,
              "lm_phase_ms_calls": {k: list(ctx_lm.kernel_time(k)) for k in
                                    ("reproj_jacobian", "semantic_jacobian", "point_prepare", "fblock", "f_allreduce", "s_zero", "s_allreduce",
                                     "schur_build", "cholesky", "cholesky_solve", "pcg", "backsub",
                                     "trial_cost")}}
        ctx_lm.close()

    if rank == 0:
        avg_j = j_ms / max(1, j_n)
        bpb = bytes_per_block(cfg["model"], cfg["track"])
        achieved = bpb * nb / (avg_j * 1e-3) / 1e9 if avg_j > 0 else 0.0
        traffic, traffic_src = pmc_traffic(args.config, "reproj_jacobian_kernel") if world == 1 else (None, None)
        warm_traffic, _ = pmc_traffic(args.config, "touch_kernel") if world == 1 else (None, None)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "residual_blocks/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * dt / args.steps,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (GenerateReconstruction restated, seed = rank for weak shards, 0 otherwise; rendered labelled plane)",
            "config": {"workload": (f"{args.config}: {cfg['desc']}" if world == 1 else
                                    f"{args.config} x{world} ({args.scaling} scaling): {cfg['desc']}"
                                    + (" per rank" if args.scaling == "weak" else " split across ranks")),
                       "cameras": cfg["images"],
                       "points": cfg["points"], "observations": cfg["points"] * cfg["track"],
                       "reprojection_blocks_rank0": nb, "semantic_samples_rank0": ns,
                       "camera_model": [k for k, v in mi_ba.MODEL_NAMES.items() if v == cfg["model"]][0],
                       "parallelism": f"point-sharded x{world}", "scaling": args.scaling},
            "roofline": {"kernel": "reproj_jacobian", "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": bpb * nb,
                         "bytes_per_block": bpb, "blocks_per_launch": nb, "avg_launch_ms": avg_j,
                         # the step reads the observations into the memory-side cache right before the
                         # kernel (linearize_warm_inputs): the kernel's rate with that read's time added
                         "input_warm_ms": w_ms / w_n if w_n else 0.0,
                         "frac_incl_input_warm": (bpb * nb / ((avg_j + (w_ms / w_n if w_n else 0.0)) * 1e-3) / 1e9
                                                  / HBM_PEAK_GBS) if avg_j > 0 else None,
                         # the warm-up's own HBM bytes (same PMC summary), and the pair's
                         "traffic_input_warm": warm_traffic,
                         "traffic_incl_input_warm": (traffic + warm_traffic) if traffic and warm_traffic else None},
            "kernels_ms": {"reproj_jacobian": avg_j, "semantic_jacobian": s_ms / max(1, s_n),
                           "input_warm": w_ms / w_n if w_n else 0.0},
            "roofline_semantic": roofline_semantic(args.config, ns, s_ms / max(1, s_n)) if ns and world == 1 else None,
            "reproj_blocks_per_s": nb * world / (avg_j * 1e-3) if avg_j > 0 else None,
            "setup_s": setup_s,
        }
        if lm:
            out.update(lm)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(opts, sc, sem, cfg, nb, ns)
            out["ba_iteration_c2"] = cpu_ba_iteration()
            # the C4 CPU iteration takes ~30 s on the 16-thread share: the committed
            # record of tools/cpu_ba_iteration.py on a GPU box, not re-measured here
            import glob
            recs = sorted(glob.glob(os.path.join(ROOT, "profiles", "*cpu_ba_iteration_c4.json")))
            if recs:
                rec = json.load(open(recs[-1]))
                rec["source"] = os.path.relpath(recs[-1], ROOT) + " (committed record, not measured in this run)"
                out["ba_iteration_c4_cpu_record"] = rec
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
