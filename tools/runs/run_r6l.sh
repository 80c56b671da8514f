# round 6 l: multi-rank rehearsal of the bench (2 ranks over gloo sharing the box's one GPU) with the
# round-6 legs (train roofline, drop-in sweep), short windows; plus the tape-timing test
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6l
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_tape.py -q -k last_tape --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
echo "rc $?" >> $O/tests.log
HSIM_BENCH_BACKEND=gloo timeout -k 10 900 python bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-episodes --cpu-steps 100 > $O/bench_2rank_gloo.log 2>&1 || exit 4
