# round 4 o: tape-launch probe (odd / small batches)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4o
timeout -k 10 300 python -u tools/probes/gpu_tape_probe.py > gpurun_out/r4o/probe.log 2>&1
