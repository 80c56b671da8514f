# round 5 d: hybrid chunk queue (whole-step items for the heaviest pairs, chunked tail of qsplit pairs):
# correctness (queue / tape / env bitwise tests) and an A/B over HSIM_QSPLIT (100000 = every pair
# chunked, the round-4 schedule), two rounds, 100 timed steps each
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5d
timeout -k 10 400 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_env.py tests/test_gpu_tape.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5d/tests.log 2>&1 || exit 2
B="python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-rollout --no-gae --train-iters 0 --no-configs --no-fp32 --no-episodes --no-tape --no-dropin"
for r in 1 2; do
  for q in 100000 1024 512 1536; do
    HSIM_QSPLIT=$q timeout -k 10 120 $B > gpurun_out/r5d/ab_q${q}_r${r}.log 2>&1 || exit 3
    echo "q=$q r=$r $(tail -1 gpurun_out/r5d/ab_q${q}_r${r}.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms_per_launch"])')" >> gpurun_out/r5d/ab.txt
  done
done
