# round 4 f: the GPU control fit with long CMA-ES runs (synthetic check first, then recorded keys)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4f
timeout -k 10 400 python -u tools/probes/gpu_trajfit.py --synthetic --intervals 56,90 --variants truth --pop 2048 --gens 5000 \
  > gpurun_out/r4f/synthetic.md 2> gpurun_out/r4f/synthetic.err || exit 5
timeout -k 10 400 python -u tools/probes/gpu_trajfit.py --synthetic --intervals 56,90 --variants truth --pop 8192 --gens 2000 \
  > gpurun_out/r4f/synthetic8k.md 2> gpurun_out/r4f/synthetic8k.err || exit 6
