# round 5 l: where the ~70 us of idle gaps inside each PPO-update minibatch (graph replay) go:
# kernel trace + memory-copy trace of the train-split probe (no counters)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5l
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r5l/prof -o tr -- python3 tools/probes/gpu_train_split.py 3 > gpurun_out/r5l/log.txt 2>&1 || exit 3
