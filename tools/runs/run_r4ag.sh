# round 4 ag: tape tests incl. tapes split over several launches (short episodes, TimeLimit truncation)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4ag
timeout -k 10 400 python -u -m pytest tests/test_gpu_tape.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r4ag/tests.log 2>&1 || exit 2
