#!/bin/bash
# One GPU session: the named stages in order, each under its own time limit;
# a test failure (pytest rc 1) does not stop the session, any crash, abort or
# timeout does.  Output under gpurun_out/<tag>/.
#   bash tools/gpu_session.sh <tag> <stage> [<stage> ...]
# stages: tests (TESTS="..." files, default the whole -m gpu suite), jac (the
# reproj_jacobian roofline decomposition in-step and back-to-back), ws (flat
# pass window summaries A/B), chol (panel schedules A/B; CHOL="k=v,k=v ..."),
# trace (rocprofv3 kernel trace of the bench command), bench (the bench line),
# jacsweep (in-step times of the tools-build Jacobian variants JACV), pcg
# (matrix-free PCG product A/B),
# prof (trace + traffic PMC of the bench step, summarized), pmcj (reproj PMC b2b vs in-step),
# pmcs (semantic PMC passes + summary), warm (linearize_warm_inputs A/B), cpuba (oracle C4 BA iteration on the box's CPU share), smoke
set -o pipefail
T=${1:?tag}
shift
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
export MI_BA_PROFILE_DIR=$PWD/gpurun_out/$T
for stage in "$@"; do
  echo "== $stage $(date +%T)"
  case $stage in
    tests)
      timeout -k 10 ${TESTS_TIMEOUT:-900} python -u -m pytest ${PYTEST_X--x} -v --timeout 400 --timeout-method thread -m gpu ${TESTS:-tests} > gpurun_out/$T/tests.log 2>&1
      rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/$T/tests.log
      [ $rc -le 1 ] || exit 1 ;;
    jac)
      timeout -k 10 300 python -u tools/ab_jacobian.py --step --variants 0,11,12 --rounds 5 --reps 5 > gpurun_out/$T/ab_jac_step.jsonl 2> gpurun_out/$T/ab_jac_step.err || exit 1
      timeout -k 10 300 python -u tools/ab_jacobian.py --variants 0,11,12 --rounds 5 --reps 5 > gpurun_out/$T/ab_jac_b2b.jsonl 2> gpurun_out/$T/ab_jac_b2b.err || exit 1
      cat gpurun_out/$T/ab_jac_step.jsonl ;;
    jacsweep)
      timeout -k 10 400 python -u tools/ab_jacobian.py --step --variants ${JACV:-0,1,2,4,30,31,32,35,39} --rounds 5 --reps 5 > gpurun_out/$T/ab_jac_sweep.jsonl 2> gpurun_out/$T/ab_jac_sweep.err || exit 1
      cat gpurun_out/$T/ab_jac_sweep.jsonl ;;
    pcg)
      timeout -k 10 500 python -u tools/ab_pcg_mf.py > gpurun_out/$T/ab_pcg_mf.jsonl 2> gpurun_out/$T/ab_pcg_mf.err || exit 1
      cat gpurun_out/$T/ab_pcg_mf.jsonl ;;
    warm)
      timeout -k 10 300 python -u tools/ab_linearize_warm.py $WARM_ARGS > gpurun_out/$T/ab_warm.jsonl 2> gpurun_out/$T/ab_warm.err || exit 1
      cat gpurun_out/$T/ab_warm.jsonl ;;
    cpuba)
      timeout -k 10 600 python -u tools/cpu_ba_iteration.py --config C4 --iters 1 > gpurun_out/$T/cpu_ba_c4.json 2> gpurun_out/$T/cpu_ba_c4.err || exit 1
      cat gpurun_out/$T/cpu_ba_c4.json ;;
    warmov)
      timeout -k 10 300 python -u tools/ab_linearize_warm.py --overlap > gpurun_out/$T/ab_warm_overlap.jsonl 2> gpurun_out/$T/ab_warm_overlap.err || exit 1
      cat gpurun_out/$T/ab_warm_overlap.jsonl ;;
    lmkeys)
      timeout -k 10 900 python -u tools/ab_lm_keys.py "" $LMKEYS > gpurun_out/$T/ab_lm_keys.jsonl 2> gpurun_out/$T/ab_lm_keys.err || exit 1
      cat gpurun_out/$T/ab_lm_keys.jsonl ;;
    ws)
      timeout -k 10 300 python -u tools/ab_semantic_ws.py > gpurun_out/$T/ab_ws.jsonl 2> gpurun_out/$T/ab_ws.err || exit 1
      cat gpurun_out/$T/ab_ws.jsonl ;;
    chol)
      timeout -k 10 600 python -u tools/ab_chol_keys.py "" $CHOL > gpurun_out/$T/ab_chol.jsonl 2> gpurun_out/$T/ab_chol.err || exit 1
      cat gpurun_out/$T/ab_chol.jsonl ;;
    prof)
      timeout -k 10 1500 bash tools/profile.sh gpurun_out/$T/prof > gpurun_out/$T/prof.log 2>&1 || { tail -5 gpurun_out/$T/prof.log; exit 1; }
      python tools/summarize_profile.py gpurun_out/$T/prof gpurun_out/$T/c4 && head -40 gpurun_out/$T/c4.md ;;
    pmcj)
      timeout -k 10 900 bash tools/pmc_jac_context.sh gpurun_out/$T/pmcctx > gpurun_out/$T/pmcctx.log 2>&1 || { tail -5 gpurun_out/$T/pmcctx.log; exit 1; }
      tail -2 gpurun_out/$T/pmcctx.log ;;
    pmcs)
      timeout -k 10 900 bash tools/pmc_semantic.sh gpurun_out/$T/pmcs > gpurun_out/$T/pmcs.log 2>&1 || { tail -5 gpurun_out/$T/pmcs.log; exit 1; }
      python tools/summarize_pmc_semantic.py gpurun_out/$T/pmcs gpurun_out/$T/c4_semantic_pmc.json && cat gpurun_out/$T/c4_semantic_pmc.json ;;
    trace)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/bench_trace -o run -- python3 bench.py --lm-iters 0 --no-cpu-baseline > gpurun_out/$T/bench_trace.log 2>&1 || exit 1
      tail -c 300 gpurun_out/$T/bench_trace.log ;;
    tracelm)
      timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/lm_trace -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/$T/lm_trace.log 2>&1 || exit 1
      tail -c 300 gpurun_out/$T/lm_trace.log ;;
    bench)
      timeout -k 10 600 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit 1
      tail -c 300 gpurun_out/$T/bench.json ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -5 gpurun_out/$T/smoke.log; exit 1; }
      tail -1 gpurun_out/$T/smoke.log ;;
    *) echo "unknown stage $stage"; exit 2 ;;
  esac
done
echo "session done $(date +%T)"
