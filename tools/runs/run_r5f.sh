# round 5 f: the full GPU suite on the current build, the default bench line, and a 2-rank
# multi-process rehearsal of bench.py (gloo, both ranks on the one GPU; the driver's 8-GPU runs use
# RCCL, one process per GPU)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5f
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5f/gputest.log 2>&1
rc=$?
echo "pytest rc $rc" >> gpurun_out/r5f/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 3; fi
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/r5f/bench.log 2>&1 || exit 4
HSIM_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 --no-episodes --no-configs --train-iters 1 > gpurun_out/r5f/bench_2rank_gloo.log 2>&1 || exit 5
