cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2c
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r2c/ppotests.log 2>&1
