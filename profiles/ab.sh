# A/B/... of builds of the product library on the fp64 headline window (bench.py sim-only leg),
# round-robin over the libraries twice: bash profiles/ab.sh <tag> <libA> <libB> [<libC> ...] [-- extra bench args]
cd $GRAFT_REPO_ROOT
TAG=$1; shift
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" == "--" ] && shift
mkdir -p gpurun_out
rm -f gpurun_out/ab_${TAG}.log
for r in 1 2; do
  for L in "${LIBS[@]}"; do
    HSIM_LIB=$L timeout -k 10 200 python -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-rollout --no-gae \
      --train-iters 0 --no-configs --no-episodes --no-fp32 "$@" > gpurun_out/ab_${TAG}_tmp.json 2> gpurun_out/ab_${TAG}_err.log || exit 9
    python -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/ab_${TAG}_tmp.json') if l.startswith('{')][-1])
print('$L', round(d['value']/1e6,4), 'M', round(d['roofline']['kernel_ms_per_launch'],4), 'ms', d['sim_stats']['warnings'], d['sim_stats']['mean_newton_iters'])" >> gpurun_out/ab_${TAG}.log
  done
done
cat gpurun_out/ab_${TAG}.log
