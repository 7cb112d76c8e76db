"""Full-size rehearsal of BASELINE's C5 on one GPU: the C4 scene (1000 OPENCV
cameras, 1M points, 10M observations, 5.0M semantic samples) point- and
pair-sharded across 2 ranks that share the card, every LM sum through gloo
(mi_ba_context_set_host_reducer: the same multi-rank code path as RCCL, whose
1-rank form tests/test_comm.py pins bitwise), with the solver bench.py uses
at N > 1: ITERATIVE_SCHUR + SCHUR_JACOBI at the default eta (0.1).  Against
the unsharded 1-rank run of the same solver and eta: 3 LM iterations, same
step counts, final cost within 1e-6 relative (north-star tolerance; the
ranks sum their shards in a different order), cameras bitwise equal across
ranks.  bundle_adjustment.cc:283-285 (ITERATIVE_SCHUR above 1000 images)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "c5_rehearsal_worker.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_c5_two_rank_pcg_matches_one_rank(gpu, tmp_path):
    one = tmp_path / "one.json"
    subprocess.run([sys.executable, WORKER, "--out", str(one)], check=True, timeout=400)
    port = _free_port()
    outs = [tmp_path / f"r{r}.json" for r in range(2)]
    procs = [subprocess.Popen([sys.executable, WORKER, "--rank", str(r), "--world", "2", "--port", str(port),
                               "--out", str(outs[r])]) for r in range(2)]
    try:
        for p in procs:
            assert p.wait(timeout=400) == 0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    ref = json.load(open(one))
    res = [json.load(open(o)) for o in outs]
    assert ref["successful"] + ref["unsuccessful"] == 3 and ref["successful"] >= 1
    for r in res:
        assert r["eta"] == ref["eta"] == 0.1
        assert abs(r["initial_cost"] - ref["initial_cost"]) <= 1e-12 * ref["initial_cost"]
        assert (r["successful"], r["unsuccessful"]) == (ref["successful"], ref["unsuccessful"])
        assert abs(r["final_cost"] - ref["final_cost"]) <= 1e-6 * ref["final_cost"], (r["final_cost"], ref["final_cost"])
        assert r["final_cost"] < r["initial_cost"]
    assert res[0]["qvec0"] == res[1]["qvec0"] and res[0]["tvec0"] == res[1]["tvec0"]
    assert res[0]["cg_iterations"] == res[1]["cg_iterations"]
    out = os.environ.get("MI_BA_PROFILE_DIR")  # the GPU session's record of the comparison
    if out:
        with open(os.path.join(out, "c5_rehearsal.json"), "w") as f:
            json.dump({"one_rank": {k: v for k, v in ref.items() if k not in ("qvec0", "tvec0")},
                       "two_ranks": [{k: v for k, v in r.items() if k not in ("qvec0", "tvec0")} for r in res]}, f,
                      indent=1)
