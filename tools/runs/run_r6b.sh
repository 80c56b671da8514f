# round 6 b: pack kernel tests + dropin leg; dynamic instruction census; PC-sampling attempt
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin_warnings.py tests/test_gpu_env.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
echo "rc $?" >> $O/tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-tape > $O/bench_dropin.log 2>&1 || exit 4
bash profiles/census.sh r6b || exit 5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 262144 --output-format csv -d $O/pcs -o pcs -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-tape --no-dropin > $O/pcs.log 2>&1
echo "pcs rc $?" >> $O/pcs.log
