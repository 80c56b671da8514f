# SURVEY 8(d) protocol on the current build: per tape T0 / T1 / T2 and seed {0, 1, 2}, reset, 1000 warm-up
# env steps, 10 000 timed -- as per-step launches and as 500-step tape calls (fp64, 4096 envs).
#   gpurun -- 'bash tools/runs/protocol.sh r6q'
TAG=${1:?usage: protocol.sh TAG}
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u bench.py --protocol --precision fp64 > $O/protocol_fp64.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py --protocol --protocol-tape --precision fp64 > $O/protocol_tape_fp64.log 2>&1 || exit 4
