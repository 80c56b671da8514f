# round 2: PGS instance parity tests + throughput probes (fp64 and fp32, staggered window)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pgs.py -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/pgs_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/probes/gpu_pgs_probe2.py > gpurun_out/pgs_probe2.log 2>&1 || exit 2
