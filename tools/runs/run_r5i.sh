# round 5 i: the fused MLP forward with 1 or 2 row blocks per wave (dynamic LDS): tests and the
# timing probe with each forced
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5i
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo.py -k fused_mlp -v -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5i/gputest.log 2>&1 || exit 3
HSIM_MLP_RB=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo.py -k fused_mlp -v -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5i/gputest_rb2.log 2>&1 || exit 4
HSIM_MLP_RB=1 timeout -k 10 300 python tools/probes/gpu_mlp2_fwd.py > gpurun_out/r5i/probe_rb1.log 2>&1 || exit 5
HSIM_MLP_RB=2 timeout -k 10 300 python tools/probes/gpu_mlp2_fwd.py > gpurun_out/r5i/probe_rb2.log 2>&1 || exit 6
timeout -k 10 300 python tools/probes/gpu_train_split.py 6 > gpurun_out/r5i/train_split.log 2>&1 || exit 7
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5i/prof_train -o train -- python3 tools/probes/gpu_train_split.py 4 > gpurun_out/r5i/train_split_prof.log 2>&1 || exit 8
