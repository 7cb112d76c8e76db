set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5a
timeout -k 10 1000 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_determinism.py tests/test_lm_semantics.py tests/test_facade.py tests/test_comm.py \
  "tests/test_gpu_scale.py::test_c2_iterative_schur_default_eta_converges_to_oracle" \
  tests/test_gpu_scale.py::test_iterative_schur_parity tests/test_gpu_scale.py::test_iterative_schur_parity_chunks \
  -s > gpurun_out/r5a/tests.log 2>&1
