# round 5 p: potential of pairing envs by predicted cost (max-of-two loss of a pair wave)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5p
timeout -k 10 300 python tools/probes/gpu_pairing_potential.py > gpurun_out/r5p/log.txt 2>&1 || exit 3
