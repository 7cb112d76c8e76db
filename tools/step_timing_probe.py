import json, os, sys, time
ROOT = "/root/repo" if os.path.exists("/root/repo") else os.getcwd()
sys.path.insert(0, os.path.join(ROOT, "semantic-bundle-adjustment-colmap_amd")); sys.path.insert(0, ROOT)
import mi_ba, bench
sc, sem = bench.build_shard(bench.CONFIGS["C4"], 0, 1)
ctx = mi_ba.Context(mi_ba.default_options(), sc, sem)
nb, _, ns = ctx.dims()
for _ in range(3):
    ctx.linearize()
ctx.synchronize()
for rnd in range(4):
    for timing in (1, 0):
        ctx.set_timing(bool(timing)); ctx.reset_kernel_times(); ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            ctx.linearize()
        ctx.synchronize()
        dt = (time.perf_counter() - t0) / 20
        print(json.dumps({"round": rnd, "timing": timing, "step_ms": round(1e3 * dt, 4)}), flush=True)
        ctx.set_timing(False)
ctx.close()
