# round 3c: cached hand-off rows + release/acquire + epoch tags + fp64 lookahead Cholesky
# (+ no MachineLICM): queue probe, full GPU suite on the new build, then A/B/C vs r3a
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probes/gpu_queue_wide_probe.py > gpurun_out/r3c_probe.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r3c_tests.log 2>&1 || exit 2
bash profiles/ab.sh r3c mujocoposelearning_amd/libhsim_base.so mujocoposelearning_amd/libhsim_la.so mujocoposelearning_amd/libhsim_nolicm.so || exit 3
bash profiles/ab.sh r3c32 mujocoposelearning_amd/libhsim_base.so mujocoposelearning_amd/libhsim_nolicm.so -- --precision fp32 || exit 4
