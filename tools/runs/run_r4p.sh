# round 4 p: pairing probe (is an env's step independent of its wave partner?)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4p
timeout -k 10 200 python -u tools/probes/gpu_pairing_probe.py 777 40 0 0 > gpurun_out/r4p/probe_stand.log 2>&1 &&
timeout -k 10 200 python -u tools/probes/gpu_pairing_probe.py 777 40 1 1 > gpurun_out/r4p/probe_kneel_full.log 2>&1
