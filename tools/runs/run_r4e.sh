# round 4 e: GPU global fit of the recorded rollout's controls -- first the synthetic check (the
# oracle's own end states from known controls), then recorded intervals, truth model only
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4e
timeout -k 10 500 python -u tools/probes/gpu_trajfit.py --synthetic --intervals 56,90,112 --variants truth --pop 2048 --gens 300 \
  > gpurun_out/r4e/synthetic.md 2> gpurun_out/r4e/synthetic.err || exit 5
timeout -k 10 500 python -u tools/probes/gpu_trajfit.py --intervals 56,90,112 --variants truth --pop 2048 --gens 300 \
  > gpurun_out/r4e/real.md 2> gpurun_out/r4e/real.err || exit 6
