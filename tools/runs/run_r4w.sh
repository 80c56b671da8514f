# round 4 w: rocprof of the tape launch beside the per-step launches (profiles/collect_tape.sh r4w)
cd $GRAFT_REPO_ROOT
bash profiles/collect_tape.sh r4w > gpurun_out/collect_r4w.log 2>&1 || exit 7
