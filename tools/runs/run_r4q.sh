# round 4 q: tape-launch determinism / first-difference probe
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4q
timeout -k 10 300 python -u tools/probes/gpu_tape_probe2.py > gpurun_out/r4q/probe.log 2>&1
